set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/pytest_gpu17.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu17.log
ARGS_FILE=tools/args_quick.txt bash tools/gpu_cmp.sh
