#!/bin/bash
# Round 6: shadow rays' first step in the pass (variant sf, TPT_SHADOW_FIRST=1) against
# the tree's library: C3 and C3 + IS, 2 interleaved reps each.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_abn.sh "C3" "cur sf" 2 --fast-extra 0 || exit 1
echo "-- env IS"
bash tools/gpu_abn.sh "C3" "cur sf" 2 --fast-extra 0 --env-is || exit 1
