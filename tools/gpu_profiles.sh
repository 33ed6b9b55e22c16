#!/bin/bash
# Round evidence: rocprof kernel stats + PMC summaries (tools/gpu_round.sh) and a bench
# line for C2 (the default bench) and C3, C3 + env IS, C4, C5, staged under
# gpurun_out/stage_profiles.  Every summary carries the profiled library's build
# identity (code-object hash), so each bench line's roofline reads the summary of
# its own build (bench.py pmc_same_build).
# Usage: bash tools/gpu_profiles.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04}
mkdir -p gpurun_out/stage_profiles
bash tools/gpu_round.sh $TAG c2 || exit 1
bash tools/gpu_round.sh $TAG c3 --config C3 || exit 1
bash tools/gpu_round.sh $TAG c3is --config C3 --env-is || exit 1
bash tools/gpu_round.sh $TAG c4 --config C4 || exit 1
bash tools/gpu_round.sh $TAG c5 --config C5 || exit 1
# bench lines read the fresh summaries (copied next to the committed ones)
cp gpurun_out/stage_profiles/*.json profiles/ 2>/dev/null
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/stage_profiles/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { echo "bench C2 failed"; exit 1; }
for c in c3 c3is c4 c5; do
  C=$(echo $c | sed 's/is$//' | tr 'a-z' 'A-Z'); x=""; [ $c = c3is ] && x="--env-is"
  timeout -k 10 600 python bench.py --config $C $x --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/stage_profiles/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; exit 1; }
done
for c in c2 c3 c3is c4 c5; do
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[2], d["value"], "Mrays/s", d["ms_per_step"], "ms", r["bound"], r["frac"], r["pmc_source"], "same build:", r.get("pmc_same_build"))' gpurun_out/stage_profiles/${TAG}_bench_$c.json $c
done
