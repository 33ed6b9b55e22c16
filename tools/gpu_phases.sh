set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in C3 C2; do
TPT_LIB=$PWD/tinypathtracer_amd/variants/prof/libtpt.so TPT_DEBUG_COUNTERS=1 \
  timeout -k 10 300 python bench.py --config $C --spp 256 --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/ph_$C.json 2> gpurun_out/ph_$C.err || { tail -5 gpurun_out/ph_$C.err; exit 1; }
echo $C; grep "tpt counters" gpurun_out/ph_$C.err | tail -1
done
