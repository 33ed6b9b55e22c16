#!/bin/bash
# Round 6, first call: the new deal/launcher tests, the tolerance-mode guard
# experiment (verdict r05 item 1), and the strong-split emulation with the cost
# deal against the interleaved one (item 3).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_deal.py tests/test_gpu_ranks.py > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u tools/fast_band.py C5 > $O/fast_band.log 2>&1 &&
for cfg in C2 C5; do
  for deal in cost interleaved; do
    timeout -k 10 300 python -u bench.py --config $cfg --emulate-ranks 8 --deal $deal --steps 1 --warmup 1 \
        --weak-extra 0 --cpu-baseline 0 --fast-extra 0 > $O/strong8_${cfg}_${deal}.json 2> $O/strong8_${cfg}_${deal}.err || exit 1
  done
done &&
for deal in cost interleaved; do
  timeout -k 10 300 python -u bench.py --config C2 --emulate-ranks 4 --deal $deal --steps 1 --warmup 1 \
      --weak-extra 0 --cpu-baseline 0 --fast-extra 0 > $O/strong4_C2_${deal}.json 2> $O/strong4_C2_${deal}.err || exit 1
done
