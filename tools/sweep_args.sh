#!/bin/bash
# Run bench.py once per argument line of $ARGS_FILE (fresh process each), print value + launch time.
while IFS= read -r line; do
  [ -z "$line" ] && continue
  out=$(timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 $line 2>/dev/null | tail -1)
  echo "[$line] $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], "Mrays/s", r["avg_launch_ms"], "ms", d["rays_per_sample"], "rays/sample")' 2>/dev/null || echo FAILED)"
done < "$ARGS_FILE"
