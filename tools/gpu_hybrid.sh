#!/bin/bash
# Hybrid lanes per pixel (render_hybrid): parity, then the strong-scaled C2 split
# (every rank's share emulated) at N = 8 and 4 with auto (hybrid), 1 and 4 lanes,
# and the heavy-tile threshold / cap at N = 8.  Usage: bash tools/gpu_hybrid.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05h}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_quad.py \
    > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
run() {   # name, args
  local o=gpurun_out/${TAG}_$1; shift
  timeout -k 10 500 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 --weak-extra 0 --config C2 \
    --scaling strong "$@" > $o.json 2> $o.err || { echo "$o FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[1].split("/")[-1], "step", d["ms_per_step"], "ms; per rank", d.get("per_rank_ms"))' $o.json
}
run n8_auto --emulate-ranks 8 || exit 1
run n8_l1 --emulate-ranks 8 --lanes-per-pixel 1 || exit 1
run n8_l4 --emulate-ranks 8 --lanes-per-pixel 4 || exit 1
run n4_auto --emulate-ranks 4 || exit 1
TPT_HYBRID_FRAC=0.3 run n8_f03 --emulate-ranks 8 || exit 1
TPT_HYBRID_FRAC=0.7 run n8_f07 --emulate-ranks 8 || exit 1
TPT_HYBRID_CAP=80 run n8_c80 --emulate-ranks 8 || exit 1
TPT_HYBRID_CAP=320 TPT_HYBRID_FRAC=0.3 run n8_c320 --emulate-ranks 8 || exit 1
