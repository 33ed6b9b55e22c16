#!/bin/bash
# Bench lines of every configuration (their roofline reads the newest committed PMC summaries).
# Usage: bash tools/gpu_benchlines.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03f}
mkdir -p gpurun_out/stage_profiles
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/stage_profiles/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { echo "bench C2 failed"; tail -5 gpurun_out/${TAG}_bench_c2.err; exit 1; }
for a in "c3:--config C3" "c3is:--config C3 --env-is" "c4:--config C4" "c5:--config C5"; do
  c=${a%%:*}; args=${a#*:}
  timeout -k 10 600 python bench.py $args --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/stage_profiles/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
done
for c in c2 c3 c3is c4 c5; do
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; v=r["limits"].get("valu_issue",{}); print(sys.argv[2], d["value"], "Mrays/s", d["ms_per_step"], "ms", r["bound"], r["frac"], "useful", v.get("useful_lane_frac"), r.get("pmc_source"))' gpurun_out/stage_profiles/${TAG}_bench_$c.json $c
done
