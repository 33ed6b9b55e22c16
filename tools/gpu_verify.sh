#!/bin/bash
# Cull verification (TPT_VERIFY_CULL build): every traversed ray of a full frame is
# re-traced in the reference's order; mismatches are logged to gpurun_out/verify_*.bin
# and counted (counters[24] in the TPT_DEBUG_COUNTERS line).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=$PWD/tinypathtracer_amd/variants/verify/libtpt.so
for spec in "C3 4096" "C3 4096 --env-is" "C2 1024" "C4 8192" "C5 256"; do
  set -- $spec
  C=$1; SPP=$2; shift 2; T=$C; [ -n "$1" ] && T=${C}is
  TPT_LIB=$LIB TPT_DEBUG_WAVES=gpurun_out/verify_$T.bin TPT_DEBUG_COUNTERS=1 timeout -k 10 400 python bench.py --config $C --spp $SPP \
    --steps 1 --warmup 0 --cpu-baseline 0 --fast-extra 0 "$@" > gpurun_out/verify_$T.json 2> gpurun_out/verify_$T.err || { echo "$T FAILED"; tail -3 gpurun_out/verify_$T.err; exit 1; }
  echo "$T $(grep 'tpt counters' gpurun_out/verify_$T.err | tail -1 | awk '{print "mismatches", $27}')"
done
