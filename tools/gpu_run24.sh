set -o pipefail
mkdir -p gpurun_out
LIBS="tinypathtracer_amd/libtpt.so tinypathtracer_amd/variants/prio3/libtpt.so tinypathtracer_amd/variants/prio5/libtpt.so" REPS=2 ARGS_FILE=tools/args_prio.txt bash tools/gpu_ab.sh > gpurun_out/ab24.log 2>&1; echo AB=$?
python tools/ab_summary.py gpurun_out/ab24.log
