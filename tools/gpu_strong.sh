#!/bin/bash
# Strong-scaling emulation on one GPU: every rank's bands of an N-way split rendered in
# turn (the step = the slowest rank's), at C2 (with the weak-scaling key) and C5.
# Usage: bash tools/gpu_strong.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03s}
mkdir -p gpurun_out
for C in C2 C5; do
for n in 1 2 4 8; do
  W="--weak-extra 1"; [ $C = C5 ] && W="--weak-extra 0"
  timeout -k 10 400 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 --scaling strong \
    --emulate-ranks $n $W > gpurun_out/${TAG}_strong_${C}_$n.json 2> gpurun_out/${TAG}_strong_${C}_$n.err || { echo "$C $n FAILED"; tail -5 gpurun_out/${TAG}_strong_${C}_$n.err; exit 1; }
  python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print(sys.argv[2], sys.argv[3], "ms/step", d["ms_per_step"], "Mrays/s", d["value"], "per-rank", d.get("per_rank_ms"), "weak", (d.get("weak") or {}).get("ms_per_step"))' gpurun_out/${TAG}_strong_${C}_$n.json $C $n
done
done
timeout -k 10 300 python bench.py --config C3 --env-is --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/${TAG}_bench_c3is.json 2> gpurun_out/${TAG}_bench_c3is.err || { tail -5 gpurun_out/${TAG}_bench_c3is.err; exit 1; }
python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read()); print("C3 IS", d["ms_per_step"], d["value"], d["roofline"]["bound"], d["roofline"]["frac"], d["roofline"]["pmc_source"])' gpurun_out/${TAG}_bench_c3is.json
