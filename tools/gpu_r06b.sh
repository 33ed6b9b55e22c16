#!/bin/bash
# Round 6: deal orders at N = 8 (C5, C2) with the probe's band costs dumped.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_deal.py > $O/tests.log 2>&1 &&
for cfg in C5 C2; do
  for deal in cost-heavy-first interleaved cost; do
    timeout -k 10 300 python -u bench.py --config $cfg --emulate-ranks 8 --deal $deal --steps 1 --warmup 1 \
        --weak-extra 0 --cpu-baseline 0 --fast-extra 0 > $O/strong8_${cfg}_${deal}.json 2> $O/strong8_${cfg}_${deal}.err || exit 1
  done
done
