set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/pytest_gpu2.log 2>&1; echo PYTEST=$?
tail -5 gpurun_out/pytest_gpu2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK; tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --spp 64 --steps 1 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_spp64.log 2>&1; echo BENCH64=$?; tail -3 gpurun_out/bench_spp64.log
