#!/bin/bash
# Four-lane visit with the leaf children's triangles in flight during the ranking
# (variants/qe, TPT_QUAD_EARLY=1) against the tree's build: parity of the variant,
# lone-walk latency, strong-scaled C2 at N = 8 (interleaved).  Usage: bash tools/gpu_quadearly.sh TAG
# (build the variant first, on the CPU side: cd tinypathtracer_amd && make -j8 OBJDIR=variants/qe/build
#  OUT=variants/qe/libtpt.so EXTRA=-DTPT_QUAD_EARLY=0 variants/qe/libtpt.so -- since round 5's final build
#  the early loads are the default, so the variant is now the "without" side)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05qe}
QE=$PWD/tinypathtracer_amd/variants/qe/libtpt.so
mkdir -p gpurun_out
TPT_LIB=$QE timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_quad.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
TPT_LIB=$QE timeout -k 10 200 python tools/step_latency.py box 2>&1 | grep "one lane"
run() {   # name, args
  local o=gpurun_out/${TAG}_$1; shift
  timeout -k 10 500 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 --weak-extra 0 --config C2 \
    --scaling strong "$@" > $o.json 2> $o.err || { echo "$o FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[1].split("/")[-1], "step", d["ms_per_step"], "ms; per rank", d.get("per_rank_ms"))' $o.json
}
TPT_LIB=$QE run qe_a --emulate-ranks 8 || exit 1
run cur_a --emulate-ranks 8 || exit 1
TPT_LIB=$QE run qe_b --emulate-ranks 8 || exit 1
run cur_b --emulate-ranks 8 || exit 1
