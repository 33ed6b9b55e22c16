#!/bin/bash
# Round 6: C5's strong-scaled shares at N = 8 (every rank emulated) with the per-chunk
# XCD rotation: the interleaved deal, the cost deal, other launch-pipeline shapes and
# 8-row bands.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06t
run() {
  local tag=$1; shift
  o=gpurun_out/r06t/$tag
  timeout -k 10 400 python bench.py --config C5 --emulate-ranks 8 --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 "$@" \
    > $o.json 2> $o.err || { echo "$tag failed"; tail -3 $o.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["ms_per_step"], d.get("per_rank_ms"))' $o.json $tag
}
run il_1
run cost --deal cost
run p4x16 --pipe-sets 4 --pipe-chunks 16
run p2x4 --pipe-sets 2 --pipe-chunks 4
run p3x16 --pipe-sets 3 --pipe-chunks 16
run rows8 --band-rows 8
run cost_p4x16 --deal cost --pipe-sets 4 --pipe-chunks 16
run il_2
