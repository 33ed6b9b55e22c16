#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for v in cur head; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/head/libtpt.so; fi
  for args in "--refill 24" "--flags 16" "--refill 24 --pipe-sets 1"; do
    i=$((i+1))
    TPT_LIB=$L timeout -k 10 300 python bench.py --config C4 --steps 1 --warmup 1 --cpu-baseline 0 $args > gpurun_out/c4ab_$i.json 2> gpurun_out/c4ab_$i.err || { echo "FAILED"; tail -3 gpurun_out/c4ab_$i.err; exit 1; }
    python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"], d["phases_ms_per_step"], d["roofline"]["avg_launch_ms"], d["roofline"]["launches_per_step"], d["local_rays"])' gpurun_out/c4ab_$i.json $v "$args"
  done
done
