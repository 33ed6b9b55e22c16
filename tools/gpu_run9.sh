set -o pipefail
mkdir -p gpurun_out
SPP=256 bash tools/sweep_variants.sh > gpurun_out/sweep13.log 2>&1; cat gpurun_out/sweep13.log
