#!/bin/bash
# LDS bank-conflict attribution on C2 (256 spp, one launch): SQ_INSTS_LDS and
# SQ_LDS_BANK_CONFLICT for the tree's library, materials in global memory
# (mtlg) and the paired 16-bit stack layout (paired); plus their bench values.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ldsattr
for v in cur mtlg paired; do
  if [ $v = cur ]; then L=$PWD/tinypathtracer_amd/libtpt.so; else L=$PWD/tinypathtracer_amd/variants/$v/libtpt.so; fi
  TPT_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU \
    -d gpurun_out/ldsattr/$v -o run --output-format csv -- python3 bench.py --spp 256 --pipe-sets 1 --steps 1 --warmup 0 --cpu-baseline 0 \
    > gpurun_out/ldsattr/$v.log 2>&1 || { echo "pmc $v failed"; tail -3 gpurun_out/ldsattr/$v.log; exit 1; }
  python3 - gpurun_out/ldsattr/$v $v <<'PY'
import csv, glob, sys
vals = {}
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(p)):
        if "k_trace" in row["Kernel_Name"]:
            vals[row["Counter_Name"]] = vals.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
print(sys.argv[2], "LDS inst %.3g  conflict cycles %.3g  per inst %.3f  lane util %.3f  VALU %.3g" % (
    vals["SQ_INSTS_LDS"], vals["SQ_LDS_BANK_CONFLICT"], vals["SQ_LDS_BANK_CONFLICT"] / vals["SQ_INSTS_LDS"],
    vals["SQ_THREAD_CYCLES_VALU"] / (64 * vals["SQ_ACTIVE_INST_VALU"]), vals["SQ_INSTS_VALU"]))
PY
done
