#!/bin/bash
# Interleaved A/B: for each repetition and argument line, run libtpt.so and every
# variant back to back (same box, same thermal state); prints one line per run.
set -o pipefail
libs=${LIBS:-"tinypathtracer_amd/libtpt.so $(ls tinypathtracer_amd/variants/*/libtpt.so 2>/dev/null)"}
for rep in $(seq ${REPS:-2}); do
  while IFS= read -r line; do
    [ -z "$line" ] && continue
    for lib in $libs; do
      name=$(basename $(dirname $lib))
      out=$(TPT_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 1 --warmup 1 --cpu-baseline 0 $line 2>/dev/null | tail -1) || exit 1
      echo "$rep $name [$line] $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"])')"
    done
  done < "${ARGS_FILE:-tools/args_one.txt}"
done
