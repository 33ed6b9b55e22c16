set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_full_v3.log 2>&1; echo BENCH=$?; tail -1 gpurun_out/bench_full_v3.log
bash tools/profile.sh r01v3 --spp 64 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/profile_v3.log 2>&1; echo PROF=$?; tail -40 gpurun_out/profile_v3.log
