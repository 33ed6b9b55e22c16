set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02d_pytest.log 2>&1; echo PYTEST=$?; tail -4 gpurun_out/r02d_pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02d_smoke.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/r02d_smoke.log; exit 1; }
tail -1 gpurun_out/r02d_smoke.log
bash tools/gpu_round.sh r02 c2 || exit 1
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/r02d_bench.json 2> gpurun_out/r02d_bench.err; echo BENCH=$?; cat gpurun_out/r02d_bench.json
