# Full GPU evidence pass: parity suite, smoke, rocprof (kernel trace + PMC) of the
# bench workload, then the bench itself (its roofline.traffic reads the PMC summary).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1; echo PYTEST=$?
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo SMOKE FAILED; tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
echo SMOKE=0; tail -1 gpurun_out/smoke_$TAG.log
bash tools/profile.sh $TAG --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/profile_$TAG.log 2>&1 || { echo PROFILE FAILED; tail -5 gpurun_out/profile_$TAG.log; exit 1; }
echo PROF=0; grep -E "avg_duration|valu_lane|wait_any_frac|l2_hit|hbm_bytes|effective" gpurun_out/profile_$TAG.log
cp gpurun_out/prof_$TAG/summary.json profiles/pmc_trace_latest.json
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err; echo BENCH=$?; tail -1 gpurun_out/bench_$TAG.json
