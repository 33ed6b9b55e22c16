#!/bin/bash
# round 5 batch: lone-wave step latency probe, C3 bisect across round 4's commits,
# strong-scaled N = 8 (C2 exact / tolerance / 8-row bands, C5 16 / 8 / 4-row bands).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/step_latency.py box > gpurun_out/r05lat_box.log 2>&1 || { tail -20 gpurun_out/r05lat_box.log; exit 1; }
grep -v '^{' gpurun_out/r05lat_box.log
bash tools/gpu_abn.sh "C3" "cur b_aba3d60 b_ca8ea4c b_dfe556e b_437c18b b_b43015b b_2704627 b_251a6ad" 3 --fast-extra 0 > gpurun_out/r05c3_ab.log 2>&1 || { tail -5 gpurun_out/r05c3_ab.log; exit 1; }
cat gpurun_out/r05c3_ab.log
bash tools/gpu_strong8.sh r05s8
