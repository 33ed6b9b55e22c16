set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu16.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu16.log
SPP=256 bash tools/sweep_variants.sh > gpurun_out/sweep16.log 2>&1; cat gpurun_out/sweep16.log
for c in C3 C4 C5; do
  timeout -k 10 300 python bench.py --config $c --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "$c FAILED"; tail -3 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_$c.json').read().strip().splitlines()[-1]); print('$c', d['value'], d['unit'], d['ms_per_step'], 'ms', d['config']['workload'])"
done
