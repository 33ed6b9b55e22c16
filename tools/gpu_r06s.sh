#!/bin/bash
# Round 6: XCD runs rotated per chunk (tree, TPT_XCD_ROT=1) against every chunk alike
# (variant norot): C5's strong-scaled shares at N = 8 and 4 (every rank emulated),
# C5 512 spp at N = 1; interleaved, 2 reps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06s
for rep in 1 2; do
for v in cur norot; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  for n in 8 4; do
    o=gpurun_out/r06s/c5n${n}_${v}_$rep
    TPT_LIB=$L timeout -k 10 400 python bench.py --config C5 --emulate-ranks $n --steps 1 --warmup 1 --weak-extra 0 \
      --cpu-baseline 0 > $o.json 2> $o.err || { echo "$o failed"; tail -3 $o.err; exit 1; }
    python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["ms_per_step"], d.get("per_rank_ms"))' $o.json "$v n$n rep$rep"
  done
  o=gpurun_out/r06s/c5n1_${v}_$rep
  TPT_LIB=$L timeout -k 10 300 python bench.py --config C5 --spp 512 --steps 1 --warmup 1 --cpu-baseline 0 --fast-extra 0 \
    > $o.json 2> $o.err || { echo "$o failed"; exit 1; }
  python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d["value"], d["ms_per_step"])' $o.json "$v n1-512spp rep$rep"
done
done
