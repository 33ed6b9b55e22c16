#!/bin/bash
# Parameter sweep: bench lines for each value of one bench flag.
# Usage: bash tools/gpu_sweep.sh "BENCH ARGS" FLAG "V1 V2 ..."
set -o pipefail
export TMPDIR=/tmp
ARGS=$1; FLAG=$2; VALS=$3
mkdir -p gpurun_out
for v in $VALS; do
  timeout -k 10 300 python bench.py $ARGS $FLAG $v --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/sweep.json 2>gpurun_out/sweep.err || { tail -5 gpurun_out/sweep.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2][:60], sys.argv[3], sys.argv[4], d["ms_per_step"], d["value"])' gpurun_out/sweep.json "$ARGS" $FLAG $v
done
