#!/bin/bash
# C5 at N = 8 (every rank emulated): launch-pipeline shapes and dispatch orders
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ab
run() {
  local tag=$1; shift
  o=gpurun_out/r06ab/$tag
  timeout -k 10 400 python bench.py --config C5 --emulate-ranks 8 --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 "$@" \
    > $o.json 2> $o.err || { echo "$tag failed"; tail -3 $o.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["ms_per_step"], d.get("per_rank_ms"))' $o.json $tag
}
run p1_hf --pipe-sets 1 --deal interleaved-heavy-first
run p1 --pipe-sets 1
run hf --deal interleaved-heavy-first
run p1_hf2 --pipe-sets 1 --deal interleaved-heavy-first
