"""Summarise tools/gpu_ab.sh output: mean value per (variant, args) and ratio to libtpt.so."""
import collections
import sys

vals = collections.defaultdict(list)
for ln in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab.log"):
    p = ln.split()
    if len(p) < 4 or not p[0].isdigit():
        continue
    args = ln[ln.index("[") + 1:ln.index("]")]
    vals[(p[1], args)].append(float(ln.split("]")[-1]))
cfgs = sorted({a for _, a in vals})
names = sorted({n for n, _ in vals}, key=lambda n: (n != "tinypathtracer_amd", n))
for a in cfgs:
    base = sum(vals[("tinypathtracer_amd", a)]) / max(1, len(vals[("tinypathtracer_amd", a)]))
    row = []
    for n in names:
        v = vals.get((n, a))
        if v:
            m = sum(v) / len(v)
            row.append(f"{n}={m:.0f} ({m / base:.3f}) [{' '.join(f'{x:.0f}' for x in v)}]")
    print(f"{a:28s} " + "  ".join(row))
