#!/bin/bash
# Refill threshold re-check on the final build: C2 (box) at 16 / 20 / 24 and C4 (tir)
# at 16 / 20, interleaved reps
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ad
for rep in 1 2 3 4; do
for spec in "C2:16" "C2:20" "C2:24" "C4:16" "C4:20"; do
  C=${spec%%:*}; R=${spec#*:}
  o=gpurun_out/r06ad/${C}_r${R}_$rep
  timeout -k 10 300 python bench.py --config $C --steps 2 --warmup 1 --cpu-baseline 0 --fast-extra 0 --refill $R > $o.json 2> $o.err || { echo "$C $R failed"; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"])' $o.json "$C refill $R rep$rep"
done
done
