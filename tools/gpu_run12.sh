set -o pipefail
mkdir -p gpurun_out
BENCH_ARGS="--config C3" SPP=256 bash tools/sweep_variants.sh > gpurun_out/sweep17.log 2>&1; cat gpurun_out/sweep17.log
TPT_DEBUG_COUNTERS=1 TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py --config C3 --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 2>&1 | grep "tpt counters"
