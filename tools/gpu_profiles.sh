#!/bin/bash
# Round evidence: rocprof kernel stats + PMC summaries (tools/gpu_round.sh) and a bench
# line for C2 (the default bench) and C3-C5, staged under gpurun_out/stage_profiles.
# Usage: bash tools/gpu_profiles.sh TAG
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out/stage_profiles
bash tools/gpu_round.sh $TAG c2 || exit 1
for C in C3 C4 C5; do
  c=$(echo $C | tr 'A-Z' 'a-z')
  bash tools/gpu_round.sh $TAG $c --config $C || exit 1
done
# bench lines read the fresh summaries (copied next to the committed ones)
cp gpurun_out/stage_profiles/*.json profiles/ 2>/dev/null
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/stage_profiles/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err || { echo "bench C2 failed"; exit 1; }
for C in C3 C4 C5; do
  c=$(echo $C | tr 'A-Z' 'a-z')
  timeout -k 10 600 python bench.py --config $C --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/stage_profiles/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $C failed"; exit 1; }
done
for c in c2 c3 c4 c5; do
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[2], d["value"], "Mrays/s", d["ms_per_step"], "ms", r["bound"], r["frac"], r["pmc_source"])' gpurun_out/stage_profiles/${TAG}_bench_$c.json $c
done
