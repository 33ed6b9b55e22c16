#!/bin/bash
for c in 16 64 128 256 1024; do
  out=$(timeout -k 10 200 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 --spp-per-launch $c 2>/dev/null | tail -1)
  echo "chunk=$c $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s", d["ms_per_step"], "ms/step", d["roofline"]["launches_per_step"], "launches")' 2>/dev/null || echo FAILED)"
done
