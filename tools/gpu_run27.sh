set -o pipefail
mkdir -p gpurun_out
SETTINGS="- TPT_PIPE_NORMAL_PRIO=1" REPS=1 ARGS_FILE=tools/args_streams.txt bash tools/gpu_ab_env.sh > gpurun_out/ab27.log 2>&1; echo AB=$?
cat gpurun_out/ab27.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 -k "pipeline or frame_batch or chunking or band" > gpurun_out/pytest_gpu27.log 2>&1; echo PYTEST=$?
tail -2 gpurun_out/pytest_gpu27.log
