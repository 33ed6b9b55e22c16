#!/bin/bash
# A/B of the product build against tinypathtracer_amd/variants/base (the previous kernel), interleaved.
# Usage: bash tools/gpu_ab3.sh TAG CONFIG REPS [extra bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-ab}; CFG=${2:-C2}; REPS=${3:-2}; shift 3
mkdir -p gpurun_out
for r in $(seq $REPS); do
for v in base prod; do
  L=""; [ $v = base ] && L="TPT_LIB=$PWD/tinypathtracer_amd/variants/base/libtpt.so"
  env $L timeout -k 10 300 python bench.py --config $CFG --steps 3 --warmup 1 --cpu-baseline 0 "$@" > gpurun_out/${TAG}_$v$r.json 2> gpurun_out/${TAG}_$v$r.err || { tail -5 gpurun_out/${TAG}_$v$r.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], d["ms_per_step"], d["value"])' gpurun_out/${TAG}_$v$r.json $v
done
done
