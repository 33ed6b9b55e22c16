#!/bin/bash
# C3 launch schedule sweep: band sets x chunks per set (pair mode, refill default).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "3 8" "3 4" "3 16" "2 8" "3 32"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --cpu-baseline 0 --pipe-sets $1 --pipe-chunks $2 > gpurun_out/sw.json 2> gpurun_out/sw.err || { echo "FAILED $cfg"; tail -3 gpurun_out/sw.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print("sets/chunks", sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["launches_per_step"])' gpurun_out/sw.json "$cfg"
done
