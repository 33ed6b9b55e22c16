set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu15.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu15.log
SPP=256 bash tools/sweep_variants.sh > gpurun_out/sweep15.log 2>&1; cat gpurun_out/sweep15.log
