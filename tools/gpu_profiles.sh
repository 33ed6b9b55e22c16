#!/bin/bash
# Round evidence: rocprof kernel stats + PMC summaries (tools/gpu_round.sh) and a bench
# line per configuration, staged under gpurun_out/stage_profiles.  Every summary
# carries the profiled library's build identity (code-object hash), so each bench
# line's roofline reads the summary of its own build (bench.py pmc_same_build).
# Usage: bash tools/gpu_profiles.sh TAG ["c2 c3 c3is c4 c5"]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r04}; CS=${2:-"c2 c3 c3is c4 c5"}
mkdir -p gpurun_out/stage_profiles
args() { case $1 in c2) echo "";; c3) echo "--config C3";; c3is) echo "--config C3 --env-is";;
         c4) echo "--config C4";; c5) echo "--config C5";; esac; }
for c in $CS; do bash tools/gpu_round.sh $TAG $c $(args $c) || exit 1; done
# bench lines read the fresh summaries (copied next to the committed ones)
cp gpurun_out/stage_profiles/*.json profiles/ 2>/dev/null
for c in $CS; do
  if [ $c = c2 ]; then extra="--steps 5 --warmup 1"; else extra="$(args $c) --steps 2 --warmup 1 --cpu-baseline 0"; fi
  timeout -k 10 600 python bench.py $extra > gpurun_out/stage_profiles/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $c failed"; exit 1; }
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[2], d["value"], "Mrays/s", d["ms_per_step"], "ms", r["bound"], r["frac"], r["pmc_source"], "same build:", r.get("pmc_same_build"))' gpurun_out/stage_profiles/${TAG}_bench_$c.json $c
done
