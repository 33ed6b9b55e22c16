set -o pipefail
mkdir -p gpurun_out
TPT_DEBUG_WAVES=gpurun_out/waves_n8.bin TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py --spp 256 --emulate-ranks 8 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/p8.log 2>&1; echo rc=$?
TPT_DEBUG_WAVES=gpurun_out/waves_n1.bin TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/p1.log 2>&1; echo rc=$?
ls -la gpurun_out/waves_n*.bin
