#!/bin/bash
# Refill-threshold sweep (tpt_params.refill): bench.py --config CFG --refill R for each R.
# Usage: bash tools/gpu_refill.sh CFG "R1 R2 .." [reps] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
CFG=${1:-C2}; RS=${2:-"16 24"}; REPS=${3:-1}; shift $(( $# < 3 ? $# : 3 )); EXTRA="$@"
mkdir -p gpurun_out
for rep in $(seq $REPS); do
for r in $RS; do
  o=gpurun_out/refill_${CFG}_${r}_$rep
  timeout -k 10 300 python bench.py --config $CFG --refill $r --steps 2 --warmup 1 --cpu-baseline 0 $EXTRA > $o.json 2> $o.err || { echo "$CFG refill $r FAILED"; tail -3 $o.err; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], "refill", sys.argv[3], d["value"], d["ms_per_step"])' $o.json $CFG $r
done
done
