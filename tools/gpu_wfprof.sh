#!/bin/bash
# Kernel-trace stats of the wavefront variant (and the megakernel beside it) on one config.
# Usage: bash tools/gpu_wfprof.sh TAG CONFIG SPP [extra bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05wp}; C=${2:-C2}; SPP=${3:-16}; shift $(( $# < 3 ? $# : 3 )); EXTRA="$@"
OUT=gpurun_out/${TAG}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/wf -o run --output-format csv -- python3 bench.py --config $C --spp $SPP --steps 1 --warmup 0 --cpu-baseline 0 --wavefront $EXTRA > $OUT/wf.log 2>&1 || { echo "wf trace failed"; tail -5 $OUT/wf.log; exit 1; }
f=$(find $OUT/wf -name '*kernel_stats.csv' | head -1); cut -d, -f1-8 "$f" | head -12
tail -1 $OUT/wf.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print("wf", d["ms_per_step"], d["value"], d["roofline"]["launches_per_step"])'
