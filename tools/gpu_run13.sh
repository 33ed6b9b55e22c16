set -o pipefail
mkdir -p gpurun_out
for a in "--config C3 --spp 256" "--config C2 --spp 256"; do
TPT_DEBUG_COUNTERS=1 TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so timeout -k 10 120 python bench.py $a --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/p.log 2>&1
grep "tpt counters" gpurun_out/p.log; python -c "import json; d=json.loads(open('gpurun_out/p.log').read().strip().splitlines()[-1]); print(d['roofline']['avg_launch_ms'])"
done
