set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/pytest_gpu3.log 2>&1; echo PYTEST=$?
tail -5 gpurun_out/pytest_gpu3.log
bash tools/variants.sh > gpurun_out/variants1.log 2>&1; cat gpurun_out/variants1.log
