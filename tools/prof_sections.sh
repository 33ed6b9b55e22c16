#!/bin/bash
# Section profile of the shading pass (TPT_PROFILE_PHASES builds under variants/): one line per variant x config.
set -o pipefail
for v in ${VARIANTS:-prof}; do
  while IFS= read -r line; do
    [ -z "$line" ] && continue
    c=$(TPT_DEBUG_COUNTERS=1 TPT_LIB=$PWD/tinypathtracer_amd/variants/$v/libtpt.so timeout -k 10 300 python bench.py --steps 1 --warmup 0 --cpu-baseline 0 $line 2>&1 | grep "tpt counters" | tail -1) || exit 1
    echo "$v [$line] $c"
  done < "${ARGS_FILE:-tools/args_one.txt}"
done
