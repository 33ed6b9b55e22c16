#!/bin/bash
# Sweep runtime knobs / library variants at reduced spp (fresh process per point).
SPP=${SPP:-64}
run() { # lib flags refill
  out=$(TPT_LIB=$PWD/$1 timeout -k 10 120 python bench.py --spp $SPP --steps 1 --warmup 1 --cpu-baseline 0 --flags $2 --refill $3 2>/dev/null | tail -1)
  echo "$1 flags=$2 refill=$3 $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s", d["roofline"]["avg_launch_ms"], "ms frac", d["roofline"]["frac"])' 2>/dev/null || echo FAILED)"
}
L=tinypathtracer_amd/libtpt.so
run $L 4 0
for r in 8 16 24 32 40 48 56; do run $L 0 $r; done
for v in tinypathtracer_amd/variants/*/libtpt.so; do run $v 0 ${REFILL:-24}; done
