#!/bin/bash
# Per-wave anatomy of rank 0 of 8 (strong-scaled C2, one 256-spp launch) with one and
# four lanes per pixel, phase-profiling build (variants/prof): occupancy timeline and the
# heaviest waves' start and life.  Usage: bash tools/gpu_quadtail.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05qt}
mkdir -p gpurun_out
for l in 1 4; do
  TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so TPT_DEBUG_WAVES=gpurun_out/${TAG}_l$l.bin TPT_DEBUG_COUNTERS=1 \
    timeout -k 10 300 python bench.py --config C2 --spp 256 --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 \
    --scaling strong --emulate-ranks 8 --emulate-rank0-only --weak-extra 0 --fast-extra 0 --lanes-per-pixel $l \
    > gpurun_out/${TAG}_l$l.json 2> gpurun_out/${TAG}_l$l.err || { echo "lanes $l FAILED"; tail -5 gpurun_out/${TAG}_l$l.err; exit 1; }
  echo "lanes $l: step $(python -c 'import sys,json; print(json.load(open(sys.argv[1]))["ms_per_step"])' gpurun_out/${TAG}_l$l.json) ms"
  python tools/wave_timeline.py gpurun_out/${TAG}_l$l.bin $([ $l = 4 ] && echo 4096 || echo 4096) | head -8
  python - gpurun_out/${TAG}_l$l.bin <<'PY'
import sys, numpy as np
d = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.float64)
d = d[d[:, 1] > 0]
t0 = d[:, 0].min()
st = (d[:, 0] - t0) / 100.0 / 1000.0; life = d[:, 1] / 100.0 / 1000.0
o = np.argsort(-life)
print("waves", len(d), "launch span ms %.1f" % (st + life).max(), "median life ms %.2f" % np.median(life))
for i in o[:6]:
    print("  heavy wave start %.1f ms life %.1f ms end %.1f steps %d passes %d rays %d" % (st[i], life[i], st[i] + life[i], d[i, 2], d[i, 3], d[i, 4]))
late = st[o[:50]]
print("  50 heaviest: start min %.1f median %.1f max %.1f ms" % (late.min(), np.median(late), late.max()))
PY
done
