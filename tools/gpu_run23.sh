set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu23.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu23.log
SETTINGS="-" REPS=2 ARGS_FILE=tools/args_refill.txt bash tools/gpu_ab_env.sh > gpurun_out/ab23.log 2>&1; echo AB=$?
cat gpurun_out/ab23.log
