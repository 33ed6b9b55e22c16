#!/bin/bash
# In-loop specular continuation (trace.hip SPECC): the -m gpu suite, then an
# interleaved A/B of TPT_FLAG_NO_SPEC_CONT on the drained launch it targets
# (strong-scaled C2, rank 0 of 8) and, with the TPT_SPEC_CONT_FULL variant
# library, at full occupancy.
# Usage: bash tools/gpu_specc.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03h}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
fi
for rep in 1 2; do
for F in 0 32; do
  timeout -k 10 300 python bench.py --config C2 --scaling strong --emulate-ranks 8 --emulate-rank0-only --weak-extra 0 \
    --steps 1 --warmup 1 --cpu-baseline 0 --flags $F > gpurun_out/${TAG}_r0of8_$F.json 2> gpurun_out/${TAG}_r0of8_$F.err \
    || { echo "r0of8 $F FAILED"; tail -5 gpurun_out/${TAG}_r0of8_$F.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print("C2 rank 0 of 8 flags", sys.argv[2], d["ms_per_step"], "ms")' gpurun_out/${TAG}_r0of8_$F.json $F
done
done
if [ -f tinypathtracer_amd/variants/specfull/libtpt.so ]; then
  bash tools/gpu_ab.sh "C2 C5" specfull 2 || exit 1
fi
