#!/bin/bash
# Wavefront variant: slot-count sweep at one config.  Usage: bash tools/gpu_wfslots.sh TAG CONFIG SPP "S1 S2 .."
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05wsl}; C=${2:-C2}; SPP=${3:-64}; SS=${4:-"0"}; shift $(( $# < 4 ? $# : 4 )); EXTRA="$@"
mkdir -p gpurun_out
for S in $SS; do
  o=gpurun_out/${TAG}_${C}_s$S
  timeout -k 10 300 python bench.py --config $C --spp $SPP --steps 1 --warmup 1 --cpu-baseline 0 --wavefront --wf-slots $S $EXTRA > $o.json 2> $o.err \
    || { echo "$C slots $S FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "slots", sys.argv[3], d["ms_per_step"], "ms", d["value"], "Mrays/s", "launches", d["roofline"]["launches_per_step"])' $o.json $C $S
done
