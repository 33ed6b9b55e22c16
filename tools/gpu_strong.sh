#!/bin/bash
# Strong-scaling emulation (rank 0's bands of an N-way split on one GPU) at C2 and
# C5, and per-wave occupancy dumps of C3 in both lane modes (profile build).
# Usage: bash tools/gpu_strong.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02s}
mkdir -p gpurun_out
for C in C2 C5; do
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --scaling strong \
    --emulate-ranks $n > gpurun_out/${TAG}_strong_${C}_$n.json 2> gpurun_out/${TAG}_strong_${C}_$n.err || { echo "$C $n FAILED"; tail -5 gpurun_out/${TAG}_strong_${C}_$n.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], sys.argv[3], "ms/step", d["ms_per_step"], "trace", d["phases_ms_per_step"]["trace"], "Mrays/s(rank0)", d["value"])' gpurun_out/${TAG}_strong_${C}_$n.json $C $n
done
done
