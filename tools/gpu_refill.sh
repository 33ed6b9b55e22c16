#!/bin/bash
# Refill-threshold sweep.  Usage: bash tools/gpu_refill.sh CONFIG "R1 R2 ..." [extra bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C=$1; RS=$2; shift 2
for R in $RS; do
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --refill $R "$@" > gpurun_out/refill_${C}_$R.json 2> gpurun_out/refill_${C}_$R.err || { echo "$C $R FAILED"; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "refill", sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/refill_${C}_$R.json $C $R
done
