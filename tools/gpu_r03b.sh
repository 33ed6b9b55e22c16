#!/bin/bash
# A15 env-IS in pair mode: parity tests, the full-size property test, C3 bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  "tests/test_gpu_parity.py::test_env_importance_sampling_parity" \
  "tests/test_gpu_parity.py::test_env_importance_sampling_full_resolution_c3" \
  "tests/test_gpu_fullsize.py::test_full_size_env_importance_sampling_c3" \
  tests/test_gpu_boundary.py > gpurun_out/r03b_pytest.log 2>&1 || { tail -40 gpurun_out/r03b_pytest.log; exit 1; }
tail -3 gpurun_out/r03b_pytest.log
for a in "--config C3" "--config C3 --env-is" "--config C3 --env-is --lanes-per-pixel 1"; do
  timeout -k 10 200 python bench.py $a --steps 1 --warmup 1 --cpu-baseline 0 >> gpurun_out/r03b_c3.jsonl 2>>gpurun_out/r03b_c3.err || { tail -5 gpurun_out/r03b_c3.err; exit 1; }
  tail -1 gpurun_out/r03b_c3.jsonl | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["config"]["workload"], d["ms_per_step"], d["value"])'
done
