#!/bin/bash
# Cull verification (TPT_VERIFY_CULL build) on the exactness scenes (synth.exactness_scene):
# every traversed ray of a 1920x1080 frame re-traced in the reference's order; mismatches
# logged to gpurun_out/verify_<scene>.bin and counted (counters[24]).  Then the GPU tests of
# those scenes.  Usage: bash tools/gpu_verify_x.sh [SPP] [SEEDS]
set -o pipefail
export TMPDIR=/tmp
SPP=${1:-1024}; SEEDS=${2:-"42 7"}
mkdir -p gpurun_out
LIB=$PWD/tinypathtracer_amd/variants/verify/libtpt.so
for sc in x1s1 x1s2 x3; do
for seed in $SEEDS; do
  TPT_LIB=$LIB TPT_DEBUG_WAVES=gpurun_out/verify_${sc}_$seed.bin TPT_DEBUG_COUNTERS=1 timeout -k 10 400 python bench.py --scene $sc \
    --spp $SPP --seed $seed --steps 1 --warmup 0 --cpu-baseline 0 --fast-extra 0 > gpurun_out/verify_${sc}_$seed.json 2> gpurun_out/verify_${sc}_$seed.err \
    || { echo "$sc FAILED"; tail -3 gpurun_out/verify_${sc}_$seed.err; exit 1; }
  echo "$sc seed $seed spp $SPP rays $(python -c 'import sys,json; print(json.loads(open(sys.argv[1]).read())["gpu_traversals"])' gpurun_out/verify_${sc}_$seed.json) $(grep 'tpt counters' gpurun_out/verify_${sc}_$seed.err | tail -1 | awk '{print "mismatches", $27}')"
done
done
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_exactness_scenes.py > gpurun_out/r05x_tests.log 2>&1 || { tail -30 gpurun_out/r05x_tests.log; exit 1; }
tail -2 gpurun_out/r05x_tests.log
