#!/bin/bash
# Cull verification of the four-lane walk (TPT_VERIFY_CULL build, variants/verify): every
# traversed ray re-traced in the reference's order, C2 and C5 with lanes_per_pixel 4, and the
# strong-scaled C2 split at N = 8 (auto: four lanes).  Usage: bash tools/gpu_verify_quad.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
LIB=$PWD/tinypathtracer_amd/variants/verify/libtpt.so
for spec in "C2 256 --lanes-per-pixel 4" "C5 16 --lanes-per-pixel 4" "C2 256 --scaling strong --emulate-ranks 8 --weak-extra 0"; do
  set -- $spec
  C=$1; S=$2; shift 2
  tag=verifyq_${C}_$(echo "$@" | tr -dc 'a-z0-9')
  TPT_LIB=$LIB TPT_DEBUG_WAVES=gpurun_out/$tag.bin TPT_DEBUG_COUNTERS=1 timeout -k 10 500 python bench.py --config $C --spp $S \
    --steps 1 --warmup 0 --cpu-baseline 0 --fast-extra 0 "$@" > gpurun_out/$tag.json 2> gpurun_out/$tag.err || { echo "$C FAILED"; tail -3 gpurun_out/$tag.err; exit 1; }
  echo "$C $S $@: $(grep 'tpt counters' gpurun_out/$tag.err | awk '{s += $27} END {print "mismatches", s, "over", NR, "renders"}')"
done
