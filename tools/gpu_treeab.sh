#!/bin/bash
# SAH tree-build variants (exact-sweep threshold, bin count) against the product build.
# Usage: bash tools/gpu_treeab.sh TAG CONFIG "variants" [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-tree}; CFG=${2:-C2}; VARS=${3:-"sw8 sw64 b16 b64"}; shift 3
mkdir -p gpurun_out
for v in prod $VARS prod; do
  L=""; [ $v != prod ] && L="TPT_LIB=$PWD/tinypathtracer_amd/variants/$v/libtpt.so"
  env $L timeout -k 10 400 python bench.py --config $CFG --steps 2 --warmup 1 --cpu-baseline 0 "$@" > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { tail -5 gpurun_out/${TAG}_$v.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], d["ms_per_step"], d["value"], d["visits_per_ray"])' gpurun_out/${TAG}_$v.json $v
done
