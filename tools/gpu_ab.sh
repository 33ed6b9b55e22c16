#!/bin/bash
# Interleaved A/B of the tree's library against a variant (default: HEAD's, built
# into tinypathtracer_amd/variants/head) on BASELINE configs.
# Usage: bash tools/gpu_ab.sh "C2 C4" [variant] [reps] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
CFGS=${1:-C2}; VAR=${2:-head}; REPS=${3:-2}; shift 3; EXTRA="$@"
mkdir -p gpurun_out
for rep in $(seq $REPS); do
for v in cur $VAR; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  line="$v"
  for C in $CFGS; do
    spp=""; [ $C = C5 ] && spp="--spp 512"
    TPT_LIB=$L timeout -k 10 300 python bench.py --config $C $spp --steps 1 --warmup 1 --cpu-baseline 0 $EXTRA \
      > gpurun_out/ab_${C}_$v.json 2> gpurun_out/ab_${C}_$v.err || { echo "$C $v FAILED"; tail -3 gpurun_out/ab_${C}_$v.err; exit 1; }
    line="$line $C $(python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(d["value"])' gpurun_out/ab_${C}_$v.json)"
  done
  echo $line
done
done
