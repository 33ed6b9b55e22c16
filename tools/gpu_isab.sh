#!/bin/bash
# C3 + IS launch-shape A/B: pair mode vs one lane per pixel (pixel pool), 4 vs 5 waves per SIMD.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_wavefront.py \
  -k "importance or env_is" > gpurun_out/isab_tests.log 2>&1 || { tail -20 gpurun_out/isab_tests.log; exit 1; }
tail -1 gpurun_out/isab_tests.log
for v in ${VARS:-cur w5}; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  for lp in ${LANES:-2 1}; do
    TPT_LIB=$L timeout -k 10 200 python bench.py --config C3 --env-is --lanes-per-pixel $lp --steps 2 --warmup 1 --cpu-baseline 0 --fast-extra 0 > gpurun_out/isab_${v}_$lp.json 2> gpurun_out/isab_${v}_$lp.err || { echo "$v $lp FAILED"; tail -3 gpurun_out/isab_${v}_$lp.err; exit 1; }
    echo "$v lanes=$lp $(python -c 'import sys,json; print(json.loads(open(sys.argv[1]).read())["ms_per_step"])' gpurun_out/isab_${v}_$lp.json) ms"
  done
done
