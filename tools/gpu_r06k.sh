#!/bin/bash
# Round 6: C5 N = 8 split (every rank) with and without XCD runs (variants/noxcd).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
for v in noxcd cur; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  TPT_LIB=$L timeout -k 10 300 python -u bench.py --config C5 --emulate-ranks 8 --steps 1 --warmup 1 --weak-extra 0 \
      --cpu-baseline 0 --fast-extra 0 > $O/c5n8_$v.json 2> $O/c5n8_$v.err || exit 1
  python3 -c "import json; d=json.load(open('$O/c5n8_$v.json')); print('C5 N=8 $v', d['ms_per_step'], d['per_rank_ms'])"
done
TPT_LIB=$PWD/tinypathtracer_amd/variants/noxcd/libtpt.so timeout -k 10 300 python -u bench.py --config C5 --spp 512 --steps 1 \
    --warmup 1 --cpu-baseline 0 --fast-extra 0 > $O/c5n1_noxcd.json 2> $O/c5n1_noxcd.err &&
python3 -c "import json; d=json.load(open('$O/c5n1_noxcd.json')); print('C5 512spp N=1 noxcd', d['value'], d['ms_per_step'])"
