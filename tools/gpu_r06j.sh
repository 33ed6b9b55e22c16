#!/bin/bash
# Round 6: one GPU, the frame's bands dispatched heaviest first (costs from a probe
# frame) against the natural order, C2 and C5 (512 spp), interleaved reps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06j
mkdir -p $O
for rep in 1 2; do
  for deal in interleaved cost-heavy-first; do
    for cfg in C2 C5; do
      spp=""; [ $cfg = C5 ] && spp="--spp 512"
      timeout -k 10 300 python -u bench.py --config $cfg $spp --deal $deal --steps 2 --warmup 1 --cpu-baseline 0 \
          --fast-extra 0 > $O/${cfg}_${deal}_$rep.json 2> $O/${cfg}_${deal}_$rep.err || exit 1
      python3 -c "import json; d=json.load(open('$O/${cfg}_${deal}_$rep.json')); print('$cfg $deal rep $rep', d['value'], d['ms_per_step'])"
    done
  done
done
