#!/bin/bash
# Tolerance-mode variants: C5 full-spp band metrics against the oracle band, and speed.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in cur fastA fastB; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  TPT_LIB=$L timeout -k 10 300 python tools/fast_band.py 2>&1 | grep "C5 band" || { echo "$v band FAILED"; exit 1; }
done
for v in cur fastA fastB; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  line="$v"
  for C in C2 C4 C5; do
    S=""; [ $C = C5 ] && S="--spp 512"
    TPT_LIB=$L timeout -k 10 300 python bench.py --config $C $S --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 --flags 64 > gpurun_out/fv_${v}_$C.json 2> gpurun_out/fv_${v}_$C.err || { echo "$v $C FAILED"; tail -3 gpurun_out/fv_${v}_$C.err; exit 1; }
    line="$line $C $(python -c 'import sys,json; print(json.loads(open(sys.argv[1]).read())["value"])' gpurun_out/fv_${v}_$C.json)"
  done
  echo "$line (tolerance mode, Mrays/s)"
done
