#!/bin/bash
# Round 6: the inner-box FMA cut's upper bound -- every slab as one FMA per bound
# (variant fmaub, TPT_FMA_SLAB_UB=1, not exact) against the tree's library:
# C2 / C5 speed, 3 interleaved reps, and SQ_INSTS_VALU per launch at C2 128 spp.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_abn.sh "C2 C5" "cur fmaub" 3 --fast-extra 0 || exit 1
mkdir -p gpurun_out/r06q
for v in cur fmaub; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  TPT_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE \
    -d gpurun_out/r06q/pmc_$v -o run --output-format csv -- python3 bench.py --config C2 --spp 128 --steps 1 --warmup 0 \
    --cpu-baseline 0 --fast-extra 0 > gpurun_out/r06q/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo done
