#!/bin/bash
# A/B of variant libraries on C2 at 1 GPU and strong-scaled rank 0 of 8 (and optional extra configs).
# Usage: bash tools/gpu_ab2.sh "var1 var2 ..." [reps]
set -o pipefail
export TMPDIR=/tmp
VARS="cur $1"; REPS=${2:-1}
mkdir -p gpurun_out
for rep in $(seq $REPS); do
for a in "--config C2" "--config C2 --scaling strong --emulate-ranks 8 --emulate-rank0-only --weak-extra 0" "--config C5 --spp 512" "--config C3"; do
for v in $VARS; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  TPT_LIB=$L timeout -k 10 300 python bench.py $a --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/ab2.json 2>gpurun_out/ab2.err || { tail -5 gpurun_out/ab2.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2][:40], sys.argv[3], d["ms_per_step"], d["value"])' gpurun_out/ab2.json "$a" $v
done
done
done
