#!/bin/bash
# Four lanes per pixel (lanes_per_pixel 4, DESIGN.md section 6 "Four lanes per ray"):
# the lone-wave walk latency, the parity tests, then the strong-scaled C2 split at
# N = 8 (every rank's share emulated on one GPU) and full-chip C2 with 1 and 4 lanes.
# Usage: bash tools/gpu_quad.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05q}
mkdir -p gpurun_out
timeout -k 10 200 python tools/step_latency.py box > gpurun_out/${TAG}_latency.log 2>&1 || { tail -5 gpurun_out/${TAG}_latency.log; exit 1; }
grep "one lane" gpurun_out/${TAG}_latency.log
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_quad.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
run() {   # name, args
  local o=gpurun_out/${TAG}_$1; shift
  timeout -k 10 500 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 --weak-extra 0 "$@" > $o.json 2> $o.err || { echo "$o FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[1].split("/")[-1], "step", d["ms_per_step"], "ms; per rank", d.get("per_rank_ms"))' $o.json
}
run C2_s8_l1 --config C2 --scaling strong --emulate-ranks 8 --lanes-per-pixel 1 || exit 1
run C2_s8_l4 --config C2 --scaling strong --emulate-ranks 8 --lanes-per-pixel 4 || exit 1
run C2_l1 --config C2 --lanes-per-pixel 1 || exit 1
run C2_l4 --config C2 --lanes-per-pixel 4 || exit 1
