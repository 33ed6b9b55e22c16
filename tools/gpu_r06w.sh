#!/bin/bash
# Round 6: which tolerance-mode approximation sets C5's tail -- the full-spp C5 band
# against the oracle (tools/fast_band.py) and the tolerance-mode speed at C2 / C5 512 spp,
# for the tree's library and variants without the hardware sin/cos (fnosc), without
# v_rcp (fnorcp) and without either (fnone: FMA contraction only).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/r06w
for v in cur fnosc fnorcp fnone; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  echo "== $v"
  TPT_LIB=$L timeout -k 10 400 python tools/fast_band.py C5 > gpurun_out/r06w/band_$v.log 2>&1 || { echo "band $v failed"; tail -3 gpurun_out/r06w/band_$v.log; exit 1; }
  grep "spp, fast (guards" gpurun_out/r06w/band_$v.log
  for C in C2 C5; do
    spp=""; [ $C = C5 ] && spp="--spp 512"
    o=gpurun_out/r06w/bench_${C}_$v
    TPT_LIB=$L timeout -k 10 300 python bench.py --config $C $spp --steps 1 --warmup 1 --cpu-baseline 0 > $o.json 2> $o.err || { echo "bench $C $v failed"; exit 1; }
    python3 -c 'import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], "exact", d["value"], "tolerance", d["tolerance_mode"]["value"])' $o.json "$C $v"
  done
done
