#!/bin/bash
# Parked-leaf batch on the drained launch (strong-scaled C2, rank 0 of 8), interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
for B in 1 2; do
  timeout -k 10 300 python bench.py --config C2 --scaling strong --emulate-ranks 8 --emulate-rank0-only --weak-extra 0 \
    --steps 1 --warmup 1 --cpu-baseline 0 --leaf-batch $B > gpurun_out/drainleaf_$B.json 2> gpurun_out/drainleaf_$B.err \
    || { echo "leaf $B FAILED"; tail -5 gpurun_out/drainleaf_$B.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print("C2 rank 0 of 8 leaf batch", sys.argv[2], d["ms_per_step"], "ms")' gpurun_out/drainleaf_$B.json $B
done
done
