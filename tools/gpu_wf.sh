#!/bin/bash
# The wavefront variant (TPT_FLAG_WAVEFRONT): its parity tests, then bench lines
# against the megakernel.  Usage: bash tools/gpu_wf.sh TAG "C2 C4" [spp] [extra bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05w}; CFGS=${2:-"C2"}; SPP=${3:-}; shift $(( $# < 3 ? $# : 3 )); EXTRA="$@"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_wavefront.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
for C in $CFGS; do
  S=""; [ -n "$SPP" ] && S="--spp $SPP"
  for v in mega wf; do
    W=""; [ $v = wf ] && W="--wavefront"
    o=gpurun_out/${TAG}_${C}_$v
    timeout -k 10 600 python bench.py --config $C $S --steps 1 --warmup 1 --cpu-baseline 0 $W $EXTRA > $o.json 2> $o.err \
      || { echo "$C $v FAILED"; tail -5 $o.err; exit 1; }
    python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], sys.argv[3], d["ms_per_step"], "ms", d["value"], "Mrays/s", d["phases_ms_per_step"]["trace"], "trace ms launches", d["roofline"]["launches_per_step"])' $o.json $C $v
  done
done
