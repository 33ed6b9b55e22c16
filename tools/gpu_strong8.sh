#!/bin/bash
# Strong-scaled N = 8, every rank's share emulated on one GPU: C2 exact and tolerance mode,
# C5 with 16-, 8- and 4-row bands (the band deal).  Usage: bash tools/gpu_strong8.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05s8}
mkdir -p gpurun_out
run() {   # name, args
  local o=gpurun_out/${TAG}_$1; shift
  timeout -k 10 500 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 --scaling strong \
    --emulate-ranks 8 --weak-extra 0 "$@" > $o.json 2> $o.err || { echo "$o FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[1].split("/")[-1], "step", d["ms_per_step"], "ms; per rank", d["per_rank_ms"])' $o.json
}
run C2_exact --config C2 || exit 1
run C2_fast --config C2 --flags 64 || exit 1
run C2_b8 --config C2 --band-rows 8 || exit 1
run C5_b16 --config C5 || exit 1
run C5_b8 --config C5 --band-rows 8 || exit 1
run C5_b4 --config C5 --band-rows 4 || exit 1
