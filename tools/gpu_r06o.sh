#!/bin/bash
# Round 6: pair mode's mid-pass exchange (a path lane whose side lane finishes in this
# pass unwinds in it): pair-mode parity, then interleaved A/B against the previous
# library (variants/base) on C3, C3 + IS, and C2 / C2 N = 4 / C5 for the other variants.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
    -k "ball or square or pair or C3 or env_is or env_importance or light" \
    tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deal.py tests/test_gpu_boundary.py \
    > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_abn.sh "C3" "cur base" 2 --fast-extra 0 > $O/ab_c3.log 2>&1 && cat $O/ab_c3.log &&
bash tools/gpu_abn.sh "C3" "cur base" 2 --fast-extra 0 --env-is > $O/ab_c3is.log 2>&1 && cat $O/ab_c3is.log &&
bash tools/gpu_abn.sh "C2 C5" "cur base" 1 --fast-extra 0 > $O/ab_c2c5.log 2>&1 && cat $O/ab_c2c5.log
