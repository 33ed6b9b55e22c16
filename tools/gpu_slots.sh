#!/bin/bash
# Slot utilisation of one C3 launch (512 spp) per lane mode: per-wave dump of the
# phase-profiling build (TPT_DEBUG_WAVES) through tools/wave_timeline.py.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for L in 1 2; do
  TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so TPT_DEBUG_WAVES=gpurun_out/slots_c3_l$L.bin \
    timeout -k 10 300 python bench.py --config C3 --spp 512 --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 \
    --lanes-per-pixel $L > gpurun_out/slots_c3_l$L.json 2> gpurun_out/slots_c3_l$L.err || { echo "C3 L$L FAILED"; tail -5 gpurun_out/slots_c3_l$L.err; exit 1; }
  echo "lanes per pixel $L"
  python tools/wave_timeline.py gpurun_out/slots_c3_l$L.bin 5120 > gpurun_out/slots_c3_l$L.txt && head -2 gpurun_out/slots_c3_l$L.txt
done
