#!/bin/bash
# Refill threshold on strong-scaled C2 (rank 0's bands of 8 and 4, emulated on one GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 8 4; do
for R in 4 8 16 24; do
  timeout -k 10 300 python bench.py --config C2 --steps 1 --warmup 1 --cpu-baseline 0 --scaling strong --emulate-ranks $n \
    --refill $R > gpurun_out/sr.json 2> gpurun_out/sr.err || { echo "FAILED $n $R"; tail -3 gpurun_out/sr.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print("N", sys.argv[2], "refill", sys.argv[3], d["ms_per_step"], "ms")' gpurun_out/sr.json $n $R
done
done
