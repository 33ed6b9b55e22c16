#!/bin/bash
# Round 6: the launch pipeline's band sets balanced by probe costs (--deal *-sets)
# against the interleaved deal: C5 N = 8, C2 N = 8 / 4 / 2 (every rank emulated), C2 N = 1.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06v
run() {
  local tag=$1; shift
  o=gpurun_out/r06v/$tag
  timeout -k 10 400 python bench.py --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 --fast-extra 0 "$@" \
    > $o.json 2> $o.err || { echo "$tag failed"; tail -3 $o.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["ms_per_step"], d["value"], d.get("per_rank_ms"))' $o.json $tag
}
run c5n8_il --config C5 --emulate-ranks 8
run c5n8_ils --config C5 --emulate-ranks 8 --deal interleaved-sets
run c5n8_cs --config C5 --emulate-ranks 8 --deal cost-sets
run c2n8_il --emulate-ranks 8
run c2n8_ils --emulate-ranks 8 --deal interleaved-sets
run c2n4_il --emulate-ranks 4
run c2n4_ils --emulate-ranks 4 --deal interleaved-sets
run c2n2_il --emulate-ranks 2
run c2n2_ils --emulate-ranks 2 --deal interleaved-sets
run c2n1_il
run c2n1_ils --deal interleaved-sets
run c5n8_ils2 --config C5 --emulate-ranks 8 --deal interleaved-sets
run c5n8_il2 --config C5 --emulate-ranks 8
