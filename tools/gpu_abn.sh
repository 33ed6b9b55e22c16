#!/bin/bash
# Interleaved A/B/... of library variants on BASELINE configs: "cur" is the
# tree's libtpt.so, any other name is tinypathtracer_amd/variants/NAME/libtpt.so.
# Usage: bash tools/gpu_abn.sh "C2 C4 C5" "cur r03 inlbox" [reps] [extra bench args]
# Prints one line per variant and rep: name, then config value pairs (Mrays/s);
# each bench JSON is kept as gpurun_out/abn_<cfg>_<variant>_<rep>.json.
set -o pipefail
export TMPDIR=/tmp
CFGS=${1:-C2}; VARS=${2:-"cur r03"}; REPS=${3:-2}; shift $(( $# < 3 ? $# : 3 )); EXTRA="$@"
mkdir -p gpurun_out
for rep in $(seq $REPS); do
for v in $VARS; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  line="$v"
  for C in $CFGS; do
    spp=""; [ $C = C5 ] && spp="--spp 512"
    o=gpurun_out/abn_${C}_${v}_$rep
    TPT_LIB=$L timeout -k 10 300 python bench.py --config $C $spp --steps 1 --warmup 1 --cpu-baseline 0 $EXTRA \
      > $o.json 2> $o.err || { echo "$C $v FAILED"; tail -3 $o.err; exit 1; }
    line="$line $C $(python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["value"])' $o.json)"
  done
  echo $line
done
done
