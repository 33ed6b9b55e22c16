#!/bin/bash
# Launch-pipeline sweep (band sets x spp chunks per set).  Usage: bash tools/gpu_pipesweep.sh CONFIG "S:C S:C ..." [extra bench args]
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=$1; PS=$2; shift 2
for P in $PS; do
  S=${P%%:*}; K=${P##*:}
  timeout -k 10 300 python bench.py --config $CFG --steps 1 --warmup 1 --cpu-baseline 0 --pipe-sets $S --pipe-chunks $K "$@" > gpurun_out/pipe_${CFG}_${S}_$K.json 2> gpurun_out/pipe_${CFG}_${S}_$K.err || { echo "$CFG $P FAILED"; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "sets:chunks", sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/pipe_${CFG}_${S}_$K.json $CFG $P
done
