#!/bin/bash
# rocprofv3 evidence for the trace kernel ("Roofline"):
#   1. kernel-trace + stats of the bench workload (dispatch durations as the bench runs them);
#   2. PMC passes, each in its own run with --kernel-trace only (never sys/runtime tracing);
#      rocprofv3 serialises dispatches while it counts, so every pass also times each
#      dispatch alone (the effective clock = GRBM_GUI_ACTIVE / 8 / that duration).
# Usage: bash tools/profile.sh TAG [bench args]   -> gpurun_out/prof_TAG/summary.json
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}; shift
ARGS=${@:---steps 1 --warmup 0 --cpu-baseline 0}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/ktrace -o run --output-format csv -- python3 bench.py $ARGS > $OUT/ktrace.log 2>&1 || { echo "kernel-trace pass failed"; exit 1; }
i=0
while read -r PASS; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $PASS -d $OUT/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done <<'PASSES'
SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_BRANCH
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
PASSES
python3 tools/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
