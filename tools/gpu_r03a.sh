#!/bin/bash
# Round-3 first GPU pass: the device-buffer boundary tests and C3 with/without env IS.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_boundary.py \
  > gpurun_out/r03a_pytest.log 2>&1 || { tail -30 gpurun_out/r03a_pytest.log; exit 1; }
tail -3 gpurun_out/r03a_pytest.log
for a in "--config C3" "--config C3 --env-is" "--config C3 --env-is --lanes-per-pixel 1"; do
  timeout -k 10 200 python bench.py $a --steps 1 --warmup 1 --cpu-baseline 0 >> gpurun_out/r03a_c3.jsonl 2>>gpurun_out/r03a_c3.err || { tail -5 gpurun_out/r03a_c3.err; exit 1; }
  tail -1 gpurun_out/r03a_c3.jsonl | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["config"]["workload"], d["ms_per_step"], d["value"])'
done
