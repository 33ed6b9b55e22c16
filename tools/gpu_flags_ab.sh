#!/bin/bash
# Interleaved A/B of two tpt_params.flags values on one config.
# Usage: bash tools/gpu_flags_ab.sh CONFIG FLAGS_A FLAGS_B [reps] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
C=$1; FA=$2; FB=$3; REPS=${4:-2}; shift 4; EXTRA="$@"
mkdir -p gpurun_out
for rep in $(seq $REPS); do
for F in $FA $FB; do
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --flags $F $EXTRA \
    > gpurun_out/fab_${C}_$F.json 2> gpurun_out/fab_${C}_$F.err || { echo "$C $F FAILED"; tail -3 gpurun_out/fab_${C}_$F.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "flags", sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/fab_${C}_$F.json $C $F
done
done
