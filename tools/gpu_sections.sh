#!/bin/bash
# Shading-pass section profile (TPT_PROFILE_PHASES build) of C2, and refill sweeps on C4/C5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in C2 C3; do
  TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so TPT_DEBUG_COUNTERS=1 timeout -k 10 300 python bench.py --config $C --spp 256 \
    --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/sec_$C.json 2> gpurun_out/sec_$C.err || { echo "$C prof FAILED"; exit 1; }
  grep "tpt counters" gpurun_out/sec_$C.err | tail -1
done
timeout -k 10 300 python bench.py --config C3 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/c3_default.json 2>/dev/null && python -c 'import json; d=json.load(open("gpurun_out/c3_default.json")); print("C3 default", d["value"], d["ms_per_step"])'
for C in C4 C5; do
for R in 16 24 32; do
  spp=""; [ $C = C5 ] && spp="--spp 256"
  timeout -k 10 300 python bench.py --config $C $spp --steps 1 --warmup 1 --cpu-baseline 0 --refill $R > gpurun_out/refill_${C}_$R.json 2> gpurun_out/refill_${C}_$R.err || { echo "$C $R FAILED"; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "refill", sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/refill_${C}_$R.json $C $R
done
done
