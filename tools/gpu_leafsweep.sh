#!/bin/bash
# Parked-leaf batch sweep.  Usage: bash tools/gpu_leafsweep.sh CONFIG "B1 B2 ..." [extra bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C=$1; BS=$2; shift 2
for B in $BS; do
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --leaf-batch $B "$@" > gpurun_out/leaf_${C}_$B.json 2> gpurun_out/leaf_${C}_$B.err || { echo "$C $B FAILED"; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "leaf batch", sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/leaf_${C}_$B.json $C $B
done
