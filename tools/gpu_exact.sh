#!/bin/bash
# Exactness + cost check: verify build at C3/C5/C4, full-size and cull tests, C2-C5 bench lines vs HEAD.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02x}
mkdir -p gpurun_out
LIB=$PWD/tinypathtracer_amd/variants/verify/libtpt.so
for spec in "C3 4096" "C5 512" "C4 8192"; do
  set -- $spec
  TPT_LIB=$LIB TPT_DEBUG_WAVES=gpurun_out/verify_$1.bin TPT_DEBUG_COUNTERS=1 timeout -k 10 400 python bench.py --config $1 --spp $2 \
    --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/verify_$1.json 2> gpurun_out/verify_$1.err || { echo "$1 FAILED"; tail -3 gpurun_out/verify_$1.err; exit 1; }
  echo "verify $1 $(grep 'tpt counters' gpurun_out/verify_$1.err | tail -1 | awk '{print "mismatches", $27}')"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_cull.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for v in cur head; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/head/libtpt.so; fi
  line=$v
  for C in C2 C3 C4 C5; do
    spp=""; [ $C = C5 ] && spp="--spp 512"
    TPT_LIB=$L timeout -k 10 300 python bench.py --config $C $spp --steps 1 --warmup 1 --cpu-baseline 0 \
      > gpurun_out/${TAG}_${C}_$v.json 2> gpurun_out/${TAG}_${C}_$v.err || { echo "$C $v FAILED"; tail -3 gpurun_out/${TAG}_${C}_$v.err; exit 1; }
    line="$line $C $(python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(d["value"])' gpurun_out/${TAG}_${C}_$v.json)"
  done
  echo $line
done
