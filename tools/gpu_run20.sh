set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu20.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu20.log
SETTINGS="- TPT_PIPE=1 TPT_PIPE=3 TPT_PIPE_CHUNKS=4 TPT_PIPE_CHUNKS=16" REPS=2 ARGS_FILE=tools/args_pipe.txt bash tools/gpu_ab_env.sh > gpurun_out/ab20.log 2>&1; echo AB=$?
cat gpurun_out/ab20.log
TPT_DEBUG_WAVES=gpurun_out/waves_box_pipe.bin TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/wboxp.log 2>&1; echo WBOX=$?
