#!/bin/bash
# Round 6: env IS searches from one-load windows (tree, TPT_ENV_WIN=1) against the
# guided search (variant nowin): C3 + IS, 3 interleaved reps; C3 once each.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_abn.sh "C3" "cur nowin" 3 --fast-extra 0 --env-is || exit 1
echo "-- no IS"
bash tools/gpu_abn.sh "C3" "cur nowin" 1 --fast-extra 0 || exit 1
