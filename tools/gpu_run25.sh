set -o pipefail
mkdir -p gpurun_out
SETTINGS="- TPT_PIPE=1 TPT_PIPE=4 TPT_PIPE_CHUNKS=12 TPT_PIPE_CHUNKS=6" REPS=2 ARGS_FILE=tools/args_pipe2.txt bash tools/gpu_ab_env.sh > gpurun_out/ab25.log 2>&1; echo AB=$?
cat gpurun_out/ab25.log
