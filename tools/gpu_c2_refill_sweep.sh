#!/bin/bash
# Refill threshold at C2's strong-scaled N = 2 shares (every rank emulated): 16 against
# the default (20 since round 6), interleaved reps
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06ae
for rep in 1 2 3; do
for R in 16 0; do
  o=gpurun_out/r06ae/n2_r${R}_$rep
  timeout -k 10 300 python bench.py --emulate-ranks 2 --steps 2 --warmup 1 --weak-extra 0 --cpu-baseline 0 --refill $R > $o.json 2> $o.err || { echo "$R failed"; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["ms_per_step"], d.get("per_rank_ms"))' $o.json "N=2 refill $R rep$rep"
done
done
