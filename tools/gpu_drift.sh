#!/bin/bash
# C5 emulation drift (verdict r04 item 5): every rank's share of an 8-way split
# rendered in turn on one GPU, in reverse order and then forward, with the GPU's
# temperature and clocks before and after each order.  If the slow shares follow
# the position in the run, it is drift; if they follow the rank, it is the deal.
# Usage: bash tools/gpu_drift.sh TAG [CONFIG]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r05d}; C=${2:-C5}
mkdir -p gpurun_out
smi() { timeout -k 5 30 rocm-smi --showtemp --showclocks --showpower > gpurun_out/${TAG}_smi_$1.txt 2>&1 || true; }
for ORD in reverse forward; do
  smi before_$ORD
  timeout -k 10 500 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --scaling strong \
    --emulate-ranks 8 --emulate-order $ORD --weak-extra 0 > gpurun_out/${TAG}_${C}_$ORD.json 2> gpurun_out/${TAG}_${C}_$ORD.err \
    || { echo "$ORD FAILED"; tail -5 gpurun_out/${TAG}_${C}_$ORD.err; exit 1; }
  smi after_$ORD
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], "per-rank", d["per_rank_ms"], "run order", d["emulate_run_ms"])' gpurun_out/${TAG}_${C}_$ORD.json $ORD
done
