#!/bin/bash
# Per-wave anatomy of a drained launch (strong-scaled C2, rank 0 of N) with the
# phase-profiling build: one launch (pipe_sets 1), counters + per-wave dump.
# Usage: bash tools/gpu_tail.sh TAG SPP "N1 N2 .."
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03t}; SPP=${2:-256}; NS=${3:-"1 8"}
mkdir -p gpurun_out
for n in $NS; do
  TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so TPT_DEBUG_WAVES=gpurun_out/${TAG}_n$n.bin TPT_DEBUG_COUNTERS=1 \
    timeout -k 10 300 python bench.py --config C2 --spp $SPP --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 \
    --scaling strong --emulate-ranks $n --emulate-rank0-only --weak-extra 0 > gpurun_out/${TAG}_n$n.json 2> gpurun_out/${TAG}_n$n.err || { echo "N=$n FAILED"; tail -5 gpurun_out/${TAG}_n$n.err; exit 1; }
  echo "N=$n"; grep "tpt counters" gpurun_out/${TAG}_n$n.err | tail -1
  python tools/wave_timeline.py gpurun_out/${TAG}_n$n.bin 5120 | head -12
done
