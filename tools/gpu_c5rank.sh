#!/bin/bash
# C5 strong-scaled N = 8: the slowest rank's share (rank 7 with 16-row bands) under other
# launch schedules.  Usage: bash tools/gpu_c5rank.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05c5r}
mkdir -p gpurun_out
for sched in "--pipe-sets 1" "--pipe-sets 2" "--pipe-sets 3" "--pipe-sets 3 --pipe-chunks 4" "--pipe-sets 3 --pipe-chunks 16" "--refill 16"; do
  o=gpurun_out/${TAG}_$(echo $sched | tr -d ' -')
  timeout -k 10 300 python bench.py --config C5 --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 --scaling strong \
    --emulate-ranks 8 --emulate-order 7 --weak-extra 0 $sched > $o.json 2> $o.err || { echo "$sched FAILED"; tail -5 $o.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "rank 7:", d["ms_per_step"], "ms")' $o.json "$sched"
done
