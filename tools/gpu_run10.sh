set -o pipefail
mkdir -p gpurun_out
TPT_DEBUG_COUNTERS=1 TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py --spp 256 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof_phases.log 2>&1; echo RC=$?
cat gpurun_out/prof_phases.log | cut -c1-400
