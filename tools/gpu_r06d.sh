#!/bin/bash
# Round 6: packed-key child sort (parity + interleaved A/B against -DTPT_PACKED_SORT=0),
# and the C5 N = 8 split with 4 x 16 and 2 x 4 launch pipelines.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
    tests/test_gpu_cull.py "tests/test_gpu_fullsize.py::test_full_size_default_order_equals_reference_order" \
    tests/test_gpu_quad.py > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
bash tools/gpu_abn.sh "C2 C4" "cur nopack" 3 --fast-extra 0 > $O/ab.log 2>&1 && cat $O/ab.log &&
for ps in "4 16" "2 4"; do
  set -- $ps
  timeout -k 10 300 python -u bench.py --config C5 --emulate-ranks 8 --deal interleaved --pipe-sets $1 --pipe-chunks $2 \
      --steps 1 --warmup 1 --weak-extra 0 --cpu-baseline 0 --fast-extra 0 > $O/c5_s$1_c$2.json 2> $O/c5_s$1_c$2.err || exit 1
  python3 -c "import json; d=json.load(open('$O/c5_s$1_c$2.json')); print('C5 N=8 sets $1 chunks $2', d['ms_per_step'], d['per_rank_ms'])"
done
