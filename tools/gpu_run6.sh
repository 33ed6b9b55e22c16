set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider > gpurun_out/pytest_gpu6.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu6.log
bash tools/sweep_variants.sh > gpurun_out/sweep3.log 2>&1; cat gpurun_out/sweep3.log
for r in 16 32; do BENCH_ARGS="--refill $r" bash tools/sweep_variants.sh 2>&1 | head -1 | sed "s/^/refill=$r /"; done
