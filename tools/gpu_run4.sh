set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x -p no:cacheprovider > gpurun_out/pytest_gpu5.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu5.log
bash tools/sweep.sh > gpurun_out/sweep1.log 2>&1; cat gpurun_out/sweep1.log
