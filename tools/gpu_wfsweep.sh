#!/bin/bash
# Wavefront variant: trace-kernel refill sweep at one config (and its PMC summaries at the
# default).  Usage: bash tools/gpu_wfsweep.sh TAG CONFIG SPP "R1 R2 .." [extra bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05ws}; C=${2:-C2}; SPP=${3:-64}; RS=${4:-"16 40"}; shift $(( $# < 4 ? $# : 4 )); EXTRA="$@"
mkdir -p gpurun_out
for R in $RS; do
  o=gpurun_out/${TAG}_${C}_r$R
  timeout -k 10 300 python bench.py --config $C --spp $SPP --steps 1 --warmup 1 --cpu-baseline 0 --wavefront --wf-refill $R $EXTRA > $o.json 2> $o.err \
    || { echo "$C refill $R FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "refill", sys.argv[3], d["ms_per_step"], "ms", d["value"], "Mrays/s")' $o.json $C $R
done
