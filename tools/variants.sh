#!/bin/bash
# Time each libtpt.so variant (fresh process each) on the bench workload at reduced spp.
SPP=${SPP:-64}
for lib in tinypathtracer_amd/libtpt.so tinypathtracer_amd/variants/*/libtpt.so; do
  for fl in ${FLAGS:-0 2}; do
    out=$(TPT_LIB=$PWD/$lib timeout -k 10 120 python bench.py --spp $SPP --steps 1 --warmup 1 --cpu-baseline 0 --flags $fl 2>/dev/null | tail -1)
    echo "$lib flags=$fl $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s", d["roofline"]["avg_launch_ms"], "ms", "frac", d["roofline"]["frac"])' 2>/dev/null || echo FAILED)"
  done
done
