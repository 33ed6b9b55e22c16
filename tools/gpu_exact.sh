#!/bin/bash
# Culling exactness round: verify build on the BASELINE frames, the full-size and
# cull GPU tests, then C2/C3/C5 bench lines of this tree against HEAD's library.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02x}
mkdir -p gpurun_out
LIB=$PWD/tinypathtracer_amd/variants/verify/libtpt.so
for spec in "C3 4096" "C5 512"; do
  set -- $spec
  TPT_LIB=$LIB TPT_DEBUG_WAVES=gpurun_out/verify_$1.bin TPT_DEBUG_COUNTERS=1 timeout -k 10 400 python bench.py --config $1 --spp $2 \
    --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/verify_$1.json 2> gpurun_out/verify_$1.err || { echo "$1 FAILED"; tail -3 gpurun_out/verify_$1.err; exit 1; }
  echo "verify $1 $(grep 'tpt counters' gpurun_out/verify_$1.err | tail -1 | awk '{print "mismatches", $27}')"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_cull.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for rep in 1 2; do
for v in cur head; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/head/libtpt.so; fi
  for C in C2 C3 C5; do
    spp=""; [ $C = C5 ] && spp="--spp 512"
    TPT_LIB=$L timeout -k 10 300 python bench.py --config $C $spp --steps 1 --warmup 1 --cpu-baseline 0 \
      > gpurun_out/${TAG}_${C}_$v.json 2> gpurun_out/${TAG}_${C}_$v.err || { echo "$C $v FAILED"; tail -3 gpurun_out/${TAG}_${C}_$v.err; exit 1; }
    python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], sys.argv[3], d["value"], d["ms_per_step"])' gpurun_out/${TAG}_${C}_$v.json $C $v
  done
done
done
