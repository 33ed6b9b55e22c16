#!/bin/bash
# Four lanes per pixel: strong-scaled C2 at N = 2, 4, 8 (every rank's share emulated)
# with 1 and 4 lanes, refill at N = 8, and a 5-wave build (variants/q5: make -j8 OBJDIR=variants/q5/build
# OUT=variants/q5/libtpt.so EXTRA=-DTPT_TRACE_WAVES_QUAD=5 variants/q5/libtpt.so in tinypathtracer_amd/).
# Usage: bash tools/gpu_quadsweep.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05qs}
mkdir -p gpurun_out
run() {   # name, args
  local o=gpurun_out/${TAG}_$1; shift
  timeout -k 10 500 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 --weak-extra 0 --config C2 \
    --scaling strong "$@" > $o.json 2> $o.err || { echo "$o FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[1].split("/")[-1], "step", d["ms_per_step"], "ms; per rank", d.get("per_rank_ms"))' $o.json
}
for n in 2 4; do
  run n${n}_l1 --emulate-ranks $n --lanes-per-pixel 1 || exit 1
  run n${n}_l4 --emulate-ranks $n --lanes-per-pixel 4 || exit 1
done
for rf in 1 2 8; do run n8_l4_refill$rf --emulate-ranks 8 --lanes-per-pixel 4 --refill $rf || exit 1; done
run n8_l4_sets1 --emulate-ranks 8 --lanes-per-pixel 4 --pipe-sets 1 || exit 1
TPT_LIB=$PWD/tinypathtracer_amd/variants/q5/libtpt.so run n8_l4_w5 --emulate-ranks 8 --lanes-per-pixel 4 || exit 1
