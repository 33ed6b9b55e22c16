set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu18.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu18.log
LIBS="tinypathtracer_amd/libtpt.so tinypathtracer_amd/variants/base/libtpt.so" REPS=2 ARGS_FILE=tools/args_tree.txt bash tools/gpu_ab.sh > gpurun_out/ab18.log 2>&1; echo AB=$?
cat gpurun_out/ab18.log
ARGS_FILE=tools/args_one.txt bash tools/prof_sections.sh > gpurun_out/sec18.log 2>&1; echo SEC=$?
cat gpurun_out/sec18.log
