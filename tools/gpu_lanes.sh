#!/bin/bash
# Lane states of the trace kernel (DESIGN.md "N1: cross-wave compaction"): the
# phase-profiling build (variants/prof, -DTPT_PROFILE_PHASES) counts, per
# traversal step, the lanes traversing / holding a finished ray that waits for
# the wave's next shading pass / without work, and the lanes each shading pass
# serves.  One 256-spp full-frame launch per config.
# Usage: [PROF_LIB=variants/NAME] bash tools/gpu_lanes.sh "C2 C5" [extra bench args]
#   (PROF_LIB: another phase-profiling build, e.g. variants/poolprof = -DTPT_TILE_POOL=1)
set -o pipefail
export TMPDIR=/tmp
CFGS=${1:-"C2 C5"}; shift; EXTRA="$@"
LIB=$PWD/tinypathtracer_amd/${PROF_LIB:-variants/prof}/libtpt.so; TAGL=$(basename ${PROF_LIB:-prof})
mkdir -p gpurun_out
for C in $CFGS; do
  TPT_LIB=$LIB TPT_DEBUG_COUNTERS=1 \
    timeout -k 10 300 python bench.py --config $C --spp 256 --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 $EXTRA \
    > gpurun_out/lanes_${TAGL}_$C.json 2> gpurun_out/lanes_${TAGL}_$C.err || { tail -5 gpurun_out/lanes_${TAGL}_$C.err; exit 1; }
  python3 - "$C" gpurun_out/lanes_${TAGL}_$C.err $TAGL <<'PY'
import sys
c = [int(x) for x in [l for l in open(sys.argv[2]) if l.startswith("tpt counters")][-1].split(":")[1].split()]
steps, passes, lt, lw, lx, lp = c[8], c[12], c[25], c[26], c[27], c[28]
tot = lt + lw + lx
print(f"{sys.argv[3]} {sys.argv[1]}: steps {steps} passes {passes} steps/pass {steps / max(passes, 1):.2f} | lane-steps: traversing "
      f"{lt / tot:.3f} waiting-for-pass {lw / tot:.3f} no-work {lx / tot:.3f} | lanes per pass {lp / max(passes, 1):.1f} | "
      f"shading ticks {c[6]} traversal ticks {c[7]} | pass sections (consume, lights/probe set-up, after, unwind, "
      f"camera, ray set-up): {' '.join(str(v) for v in c[17:23])}")
PY
done
