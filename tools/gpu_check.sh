#!/bin/bash
# GPU check of the current tree: the -m gpu suite, then bench lines at C2 (default),
# C3 and C5.  Every GPU step has its own time limit; the first failure ends the call.
# Usage: bash tools/gpu_check.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -3 gpurun_out/${TAG}_pytest.log
fi
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/${TAG}_bench_c2.json 2> gpurun_out/${TAG}_bench_c2.err \
  || { echo "bench C2 failed"; tail -5 gpurun_out/${TAG}_bench_c2.err; exit 1; }
for C in C3 C5; do
  c=$(echo $C | tr 'A-Z' 'a-z')
  timeout -k 10 400 python bench.py --config $C --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err \
    || { echo "bench $C failed"; tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
done
for c in c2 c3 c5; do
  python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d["value"], "Mrays/s", d["ms_per_step"], "ms/step")' gpurun_out/${TAG}_bench_$c.json $c
done
