#!/bin/bash
# Round 6: mid-pass exchange in every pair variant (cur) / only with env IS (midis) /
# round-start (base), C3, 3 interleaved reps.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
bash tools/gpu_abn.sh "C3" "cur midis base" 3 --fast-extra 0
