#!/bin/bash
# Refill-threshold sweep on C3 (tail-bound) and C2 (throughput-bound).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in C3; do
for R in 2 4 6 8 12; do
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --refill $R > gpurun_out/refill_${C}_$R.json 2> gpurun_out/refill_${C}_$R.err || { echo "$C $R FAILED"; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "refill", sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/refill_${C}_$R.json $C $R
done
done
