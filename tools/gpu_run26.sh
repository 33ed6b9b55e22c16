set -o pipefail
mkdir -p gpurun_out
SETTINGS="- TPT_PIPE=1" REPS=1 ARGS_FILE=tools/args_streams.txt bash tools/gpu_ab_env.sh > gpurun_out/ab26.log 2>&1; echo AB=$?
cat gpurun_out/ab26.log
for n in 1 2 4 8; do timeout -k 10 300 python bench.py --emulate-ranks $n --steps 1 --warmup 1 --cpu-baseline 0 2>/dev/null | tail -1 | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print("emulate", d["config"]["parallelism"], d["value"], d["ms_per_step"])' || exit 1; done
