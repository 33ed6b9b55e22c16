set -o pipefail
mkdir -p gpurun_out
for lib in tinypathtracer_amd/libtpt.so tinypathtracer_amd/variants/abs/libtpt.so; do
  echo "== $lib"
  TPT_LIB=$PWD/$lib ARGS_FILE=tools/args_scale.txt bash tools/sweep_args.sh 2>&1 | grep -v "band-rows"
  TPT_LIB=$PWD/$lib timeout -k 10 200 python bench.py --config C3 --spp 256 --steps 1 --warmup 1 --cpu-baseline 0 2>/dev/null | python -c 'import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print("C3", d["value"])'
done
