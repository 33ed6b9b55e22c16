#!/bin/bash
# Evidence for the env configurations (C3 and C3 + env IS): rocprof kernel stats + PMC
# summaries (tools/gpu_round.sh) staged under gpurun_out/stage_profiles, then their
# bench lines (whose roofline reads those summaries).
# Usage: bash tools/gpu_envprof.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03g}
mkdir -p gpurun_out/stage_profiles
bash tools/gpu_round.sh $TAG c3 --config C3 || exit 1
bash tools/gpu_round.sh $TAG c3is --config C3 --env-is || exit 1
cp gpurun_out/stage_profiles/*.json profiles/ 2>/dev/null
timeout -k 10 600 python bench.py --config C3 --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/stage_profiles/${TAG}_bench_c3.json 2> gpurun_out/${TAG}_bench_c3.err || { echo "bench C3 failed"; exit 1; }
timeout -k 10 600 python bench.py --config C3 --env-is --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/stage_profiles/${TAG}_bench_c3is.json 2> gpurun_out/${TAG}_bench_c3is.err || { echo "bench C3 IS failed"; exit 1; }
for c in c3 c3is; do
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[2], d["value"], "Mrays/s", d["ms_per_step"], "ms", r["bound"], r["frac"], r["pmc_source"])' gpurun_out/stage_profiles/${TAG}_bench_$c.json $c
done
