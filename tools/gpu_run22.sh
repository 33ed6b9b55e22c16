set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu22.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu22.log
SETTINGS="- TPT_PIPE=1 TPT_PIPE=3" REPS=2 ARGS_FILE=tools/args_pipe.txt bash tools/gpu_ab_env.sh > gpurun_out/ab22.log 2>&1; echo AB=$?
cat gpurun_out/ab22.log
REFILLS="16 20 24" SPP=1024 bash tools/sweep_refill.sh > gpurun_out/refill22.log 2>&1; echo REFILL=$?
cat gpurun_out/refill22.log
