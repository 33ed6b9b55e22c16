#!/bin/bash
# Interleaved A/B over environment settings of one library: for each repetition
# and argument line, run bench.py once per setting in $SETTINGS ("-" = none),
# back to back; prints value (Mrays/s) and the kernel's 4-wide visits per ray.
set -o pipefail
SETTINGS=${SETTINGS:-"- TPT_WIDE_TREE=lbvh"}
for rep in $(seq ${REPS:-2}); do
  while IFS= read -r line; do
    [ -z "$line" ] && continue
    for st in $SETTINGS; do
      if [ "$st" = "-" ]; then envs=(); else envs=("$st"); fi
      out=$(env "${envs[@]}" timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 $line 2>/dev/null | tail -1) || exit 1
      echo "$rep $st [$line] $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); s=d.get("stats",{}); print(d["value"], d["roofline"]["bytes_per_launch"])')"
    done
  done < "${ARGS_FILE:-tools/args_one.txt}"
done
