#!/bin/bash
# round 5: tolerance-mode tests + bench lines (exact with the tolerance key), then the
# wavefront variant's tests, slot sweep and PMC summaries.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_tolerance.py \
  > gpurun_out/r05a_tol.log 2>&1 || { tail -30 gpurun_out/r05a_tol.log; exit 1; }
grep -E "passed|failed|tolerance mode" gpurun_out/r05a_tol.log | tail -8
for C in C2 C4; do
  timeout -k 10 600 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/r05a_bench_$C.json 2> gpurun_out/r05a_bench_$C.err || { tail -5 gpurun_out/r05a_bench_$C.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "exact", d["ms_per_step"], d["value"], "tolerance", d.get("tolerance_mode"))' gpurun_out/r05a_bench_$C.json $C
done
bash tools/gpu_wf.sh r05w4 "C2" 64 && bash tools/gpu_wfslots.sh r05wsl C2 64 "1048576 524288" && bash tools/gpu_wfpmc.sh r05wpmc2
