#!/bin/bash
# refill threshold sweep on the bench workload (reduced spp)
SPP=${SPP:-256}
for r in ${REFILLS:-16 20 24 28 32 40}; do
  out=$(timeout -k 10 120 python bench.py --spp $SPP --steps 1 --warmup 1 --cpu-baseline 0 --refill $r 2>/dev/null | tail -1)
  echo "refill=$r $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s")' 2>/dev/null || echo FAILED)"
done
