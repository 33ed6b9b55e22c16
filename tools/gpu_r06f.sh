#!/bin/bash
# Round 6: packed fp32 slab products (variants/pk, -DTPT_PK_SLAB=1) against the tree's library.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
bash tools/gpu_abn.sh "C2 C4 C5" "cur pk" 3 --fast-extra 0 > $O/ab.log 2>&1; rc=$?; cat $O/ab.log; exit $rc
