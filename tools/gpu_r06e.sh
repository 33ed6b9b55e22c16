#!/bin/bash
# Round 6: launch-pipeline shape for strong-scaled shares of about one million pixels
# (C2 N = 2, every rank; C5 N = 8, every rank) and C2 N = 4.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
for ps in "3 8" "2 4" "2 8" "4 16" "4 8"; do
  set -- $ps
  timeout -k 10 300 python -u bench.py --config C2 --emulate-ranks 2 --deal interleaved --pipe-sets $1 --pipe-chunks $2 \
      --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 --fast-extra 0 > $O/c2n2_s$1_c$2.json 2> $O/c2n2_s$1_c$2.err || exit 1
  python3 -c "import json; d=json.load(open('$O/c2n2_s$1_c$2.json')); print('C2 N=2 sets $1 chunks $2', d['ms_per_step'], d['per_rank_ms'])"
done
for ps in "3 8" "2 4" "4 16"; do
  set -- $ps
  timeout -k 10 300 python -u bench.py --config C2 --emulate-ranks 4 --deal interleaved --pipe-sets $1 --pipe-chunks $2 \
      --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 --fast-extra 0 > $O/c2n4_s$1_c$2.json 2> $O/c2n4_s$1_c$2.err || exit 1
  python3 -c "import json; d=json.load(open('$O/c2n4_s$1_c$2.json')); print('C2 N=4 sets $1 chunks $2', d['ms_per_step'], d['per_rank_ms'])"
done
for ps in "2 8" "3 8"; do
  set -- $ps
  timeout -k 10 300 python -u bench.py --config C5 --emulate-ranks 8 --deal interleaved --pipe-sets $1 --pipe-chunks $2 \
      --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 --fast-extra 0 > $O/c5n8_s$1_c$2.json 2> $O/c5n8_s$1_c$2.err || exit 1
  python3 -c "import json; d=json.load(open('$O/c5n8_s$1_c$2.json')); print('C5 N=8 sets $1 chunks $2', d['ms_per_step'], d['per_rank_ms'])"
done
