#!/bin/bash
# The GPU parity suites with the wavefront variant forced on every render
# (TPT_TEST_FORCE_FLAGS=32, TPT_FLAG_WAVEFRONT).  Usage: bash tools/gpu_wfsuite.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05wfs}
mkdir -p gpurun_out
TPT_TEST_FORCE_FLAGS=32 timeout -k 10 1000 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_integration.py tests/test_ref_hot_kat.py \
  "tests/test_gpu_fullsize.py::test_full_spp_band_matches_oracle" -k "not fast" > gpurun_out/${TAG}.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}.log | sed 's/ PASSED.*/ PASSED/' | awk '{print $NF}' | sort | uniq -c
grep -E "FAILED|Error" gpurun_out/${TAG}.log | head -20
tail -3 gpurun_out/${TAG}.log
exit $rc
