#!/bin/bash
# 1-GPU emulation of the N-rank bench (rank 0's share of an N-way split) for
# both scaling modes, box 1080p at the given spp.  Usage: bash tools/gpu_scale.sh SPP
set -o pipefail
SPP=${1:-256}
for mode in weak strong; do
for n in 1 2 4 8; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --spp $SPP --cpu-baseline 0 --scaling $mode \
    --emulate-ranks $n > gpurun_out/scale_${mode}_$n.json 2> gpurun_out/scale_${mode}_$n.err || { echo "$mode $n FAILED"; tail -5 gpurun_out/scale_${mode}_$n.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], sys.argv[3], "ms/step", d["ms_per_step"], "trace", d["phases_ms_per_step"]["trace"], "Mrays/s(rank0)", d["value"])' gpurun_out/scale_${mode}_$n.json $mode $n
done
done
