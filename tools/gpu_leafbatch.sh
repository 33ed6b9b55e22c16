#!/bin/bash
# Parked-leaf batch sweep (tpt_params.leaf_batch).  Usage: bash tools/gpu_leafbatch.sh CONFIG "K1 K2 ..." [extra bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
C=$1; KS=$2; shift 2
for K in $KS; do
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --leaf-batch $K "$@" > gpurun_out/lb_${C}_$K.json 2> gpurun_out/lb_${C}_$K.err || { echo "$C $K FAILED"; tail -3 gpurun_out/lb_${C}_$K.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "leaf_batch", sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/lb_${C}_$K.json $C $K
done
