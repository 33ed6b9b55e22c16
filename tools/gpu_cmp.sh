# Compare libtpt.so against every variant on the argument lines of $ARGS_FILE.
set -o pipefail
mkdir -p gpurun_out
for lib in tinypathtracer_amd/libtpt.so tinypathtracer_amd/variants/*/libtpt.so; do
  echo "== $lib"
  TPT_LIB=$PWD/$lib bash tools/sweep_args.sh
done
