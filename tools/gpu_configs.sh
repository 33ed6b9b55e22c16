#!/bin/bash
# GPU evidence at the BASELINE configurations C3-C5 at their stated
# sizes: rocprof kernel stats + PMC summary (tools/gpu_round.sh) and a bench line each.
# Usage: bash tools/gpu_configs.sh TAG [C3 C4 C5]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}; shift
CFGS=${@:-C3 C4 C5}
for C in $CFGS; do
  c=$(echo $C | tr 'A-Z' 'a-z')
  echo "== $C $(date +%T)"
  bash tools/gpu_round.sh $TAG $c --config $C || exit 1
  timeout -k 10 900 python bench.py --config $C --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err || { echo "bench $C failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); r=d["roofline"]; print(sys.argv[2], d["value"], "Mrays/s", d["ms_per_step"], "ms/step", r["bound"], r["frac"], "rays/sample", d["rays_per_sample"])' gpurun_out/${TAG}_bench_$c.json $C
done
