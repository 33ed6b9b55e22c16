#!/bin/bash
# Round 6: launch-pipeline shape for the strong-scaled shares (C5 ranks 7 and 0 of 8;
# C2 every rank of 8), interleaved deal.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
for ps in 3 2 4 1; do
  for pc in 8 16 4; do
    timeout -k 10 200 python -u bench.py --config C5 --emulate-ranks 8 --emulate-order 7,0 --deal interleaved \
        --pipe-sets $ps --pipe-chunks $pc --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 --fast-extra 0 \
        > $O/c5_s${ps}_c${pc}.json 2> $O/c5_s${ps}_c${pc}.err || exit 1
    python3 -c "import json; d=json.load(open('$O/c5_s${ps}_c${pc}.json')); print('C5 sets $ps chunks $pc', d['per_rank_ms'], d['emulate_run_ms'])"
  done
done
for ps in 3 2 4; do
  for pc in 8 16 4; do
    timeout -k 10 200 python -u bench.py --config C2 --emulate-ranks 8 --deal interleaved \
        --pipe-sets $ps --pipe-chunks $pc --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 --fast-extra 0 \
        > $O/c2_s${ps}_c${pc}.json 2> $O/c2_s${ps}_c${pc}.err || exit 1
    python3 -c "import json; d=json.load(open('$O/c2_s${ps}_c${pc}.json')); print('C2 sets $ps chunks $pc', d['ms_per_step'], d['per_rank_ms'])"
  done
done
