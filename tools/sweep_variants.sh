#!/bin/bash
# Time each variant library on the bench workload (reduced spp), fresh process each.
SPP=${SPP:-64}
for lib in tinypathtracer_amd/libtpt.so tinypathtracer_amd/variants/*/libtpt.so; do
  out=$(TPT_LIB=$PWD/$lib timeout -k 10 120 python bench.py --spp $SPP --steps 1 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS} 2>/dev/null | tail -1)
  echo "$lib $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s", d["roofline"]["avg_launch_ms"], "ms frac", d["roofline"]["frac"])' 2>/dev/null || echo FAILED)"
done
