#!/bin/bash
# Per-phase scene-build times (TPT_BUILD_TIMING) for C5: synchronous and asynchronous
# builds at the default build threads, and a synchronous build with THREADS2 threads.
# Usage: bash tools/gpu_buildtime.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-bt}
mkdir -p gpurun_out
run() {   # name, extra args
  TPT_BUILD_TIMING=1 timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --cpu-baseline 0 $2 \
    > gpurun_out/${TAG}_c5_$1.json 2> gpurun_out/${TAG}_c5_$1.err || { tail -5 gpurun_out/${TAG}_c5_$1.err; exit 1; }
  echo "== $1"; tail -12 gpurun_out/${TAG}_c5_$1.err
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(d["phases_ms_per_step"], d.get("build_threads"), d["ms_per_step"])' gpurun_out/${TAG}_c5_$1.json
}
run async "--async-build 1"
run sync "--async-build 0"
run sync_t${THREADS2:-2} "--async-build 0 --build-threads ${THREADS2:-2}"
