set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu19.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu19.log
LIBS="tinypathtracer_amd/libtpt.so tinypathtracer_amd/variants/pf/libtpt.so tinypathtracer_amd/variants/base/libtpt.so" REPS=2 ARGS_FILE=tools/args_tree.txt bash tools/gpu_ab.sh > gpurun_out/ab19.log 2>&1; echo AB=$?
python tools/ab_summary.py gpurun_out/ab19.log
TPT_DEBUG_WAVES=gpurun_out/waves_box.bin TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/wbox.log 2>&1; echo WBOX=$?
TPT_DEBUG_WAVES=gpurun_out/waves_c3.bin TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py --config C3 --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/wc3.log 2>&1; echo WC3=$?
REFILLS="16 20 24 28 32" SPP=256 bash tools/sweep_refill.sh > gpurun_out/refill19.log 2>&1; echo REFILL=$?
cat gpurun_out/refill19.log
