#!/bin/bash
# Round 6: the env lookup's double-precision fallback out of line in the inlined (env IS)
# lookups -- IS variants' spills 28 -> 8 -- against the previous inlining (variants/nocold),
# C3 + IS and C3; then the env-IS parity cases.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
bash tools/gpu_abn.sh "C3" "cur nocold" 2 --fast-extra 0 --env-is > $O/ab_is.log 2>&1 && cat $O/ab_is.log &&
bash tools/gpu_abn.sh "C3" "cur nocold" 2 --fast-extra 0 > $O/ab.log 2>&1 && cat $O/ab.log &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu -k "env_is or env_importance or C3" \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_wavefront.py > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; exit $rc
