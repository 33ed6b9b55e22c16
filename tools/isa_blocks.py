#!/usr/bin/env python3
"""Per-basic-block instruction classes of one kernel in a gfx950 .s dump.

usage: isa_blocks.py kernel.s [--loops]

Prints, for every block: VALU / SALU / VMEM / SMEM / LDS / branch counts and its
successors, so a loop's per-iteration cost can be summed by hand (DESIGN.md
"ISA breakdown").  Dump a kernel with
  hipcc ... --cuda-device-only -S trace.hip -o trace.s
and cut one function out of it (from its label to the next .Lfunc_end).
"""
import re
import sys
from collections import OrderedDict


def classify(op):
    if op.startswith("v_"):
        if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
            return "valu"   # issued on the VALU too
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "br"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def parse(path):
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = {"n": {}, "succ": [], "ops": []}
    prev_falls = True
    for line in open(path):
        s = line.split(";")[0].rstrip()
        if not s.strip():
            continue
        m = re.match(r"^(\.LBB\w+|\w+):", s)
        if m:
            name = m.group(1)
            if prev_falls and cur is not None:
                blocks[cur]["succ"].append(name)
            cur = name
            blocks.setdefault(cur, {"n": {}, "succ": [], "ops": []})
            prev_falls = True
            continue
        t = s.strip()
        if t.startswith("."):
            continue
        op = t.split()[0]
        c = classify(op)
        b = blocks[cur]
        b["n"][c] = b["n"].get(c, 0) + 1
        b["ops"].append(t)
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = t.split()[-1]
            b["succ"].append(tgt)
            prev_falls = op != "s_branch"
        if op == "s_endpgm":
            prev_falls = False
    return blocks


def main():
    blocks = parse(sys.argv[1])
    tot = {}
    for name, b in blocks.items():
        n = b["n"]
        for k, v in n.items():
            tot[k] = tot.get(k, 0) + v
        print(f"{name:14s} valu {n.get('valu',0):4d} salu {n.get('salu',0):3d} vmem {n.get('vmem',0):3d} "
              f"smem {n.get('smem',0):3d} lds {n.get('lds',0):3d} wait {n.get('wait',0):3d} br {n.get('br',0):2d}"
              f"  -> {' '.join(b['succ'])}")
    print("total", tot)


if __name__ == "__main__":
    main()
