#!/usr/bin/env python3
"""Static instruction counts of one k_trace variant by source section
("ISA breakdown").

usage: isa_sections.py dump_g.s KERNEL_SYMBOL trace.hip [trace_dev.hpp]

dump_g.s: a `hipcc -O3 -g --cuda-device-only -S` dump of trace.hip; the
kernel is read from its label to the next .Lfunc_end.  Every instruction is
charged by its .loc and inlining chain: the outermost device helper on the
chain that owns a section (trace_dev.hpp functions: the 4-wide visit, the leaf
test, the BSDF sample, ...) decides, so the slab test inlined into the probe
pre-test counts as the pre-test; otherwise the k_trace line the chain starts
from, through the kernel's section markers (TPT_SEC(k), the traversal loop).
Counts are static (code size per section); per-visit costs follow because a
wave runs a section's straight-line code once per iteration in which any lane
takes it.
"""
import os
import re
import sys
from collections import defaultdict


def classify(op):
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith("scratch_"):
        return "scratch"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return None


HELPERS = [("box_hit", "trav: binary visit"), ("inner_visit", "trav: binary visit"),
           ("slab_minmax", "trav: 4-wide visit"), ("inner_visit4_q", "trav: 4-wide visit"),
           ("inner_visit4", "trav: 4-wide visit"),
           ("tri_core", "trav: leaf test"), ("cull_slack", "trav: leaf test"),
           ("leaf_test_q", "trav: leaf test"), ("leaf_test", "trav: leaf test"),
           ("sliver_pass", "pass: sliver re-test"),
           ("new_direction", "pass: BSDF sample (getNewDirection)"),
           ("probe_misses_emitters", "pass: probe pre-test"),
           ("trav_begin", "pass: ray set-up (trav_begin)"), ("grazing", "pass: grazing test"),
           ("light_sample", "pass: delta lights"), ("env_lookup_inl", "pass: env lookup"),
           ("env_is_sample", "pass: env IS"), ("emit_probe_inline", "pass: inline emitter test")]


class Src:
    def __init__(self, path):
        self.lines = open(path).read().split("\n")

    def find(self, pat, start=0):
        for i in range(start, len(self.lines)):
            if re.search(pat, self.lines[i]):
                return i + 1
        raise SystemExit(f"pattern not found: {pat}")

    def func(self, name):   # a function's line range: its signature to the closing brace at column 0
        a = self.find(r"__forceinline__ .*\b" + name + r"\(")
        b = a
        while not self.lines[b - 1].startswith("}"):
            b += 1
        return a, b


def helper_ranges(src):
    rng = []
    for name, sec in HELPERS:
        try:
            a, b = src.func(name)
        except SystemExit:   # (a helper this file does not hold)
            continue
        rng.append((a, b, sec))
    return rng


def kernel_ranges(src):
    k = src.find(r"^void k_trace\(")
    loop_top = src.find(r"^    for \(;;\) \{", k)
    done = src.find(r"if \(in_pass\) \{", loop_top + 1)
    s = [src.find(rf"TPT_SEC\({i}\)", done) for i in range(1, 7)]
    tl = src.find(r"const int thr = refill;", s[5])
    leafdec = src.find(r"const unsigned long long hb = __ballot\(has\);", tl)
    tend = src.find(r"if \(ts == TS_TRAV && r.node < 0 && r.pend < 0\) ts = TS_DONE;", leafdec)
    kend = src.find(r"^}", tend)
    return [(k, loop_top, "kernel prologue"), (loop_top, done, "pass: sliver / probe pass-2 hand-over"),
            (done, s[0], "pass: consume (hit prelude, env miss)"), (s[0], s[1], "pass: lights / probe set-up"),
            (s[1], s[2], "pass: after (next bounce)"), (s[2], s[3], "pass: unwind"), (s[3], s[4], "pass: camera ray"),
            (s[4], s[5], "pass: ray set-up (trav_begin)"), (s[5], tl, "pass: exit test"),
            (tl, leafdec, "trav: loop control, stack pop, leaf park"),
            (leafdec, tend, "trav: leaf-test decision"), (tend, tend + 2, "trav: loop control, stack pop, leaf park"),
            (tend + 3, kend, "kernel epilogue (state write-back, counters)")]


def innermost(rng, ln, default="other"):
    sec, best = default, None
    for a, b, name in rng:
        if a <= ln <= b and (best is None or b - a < best):
            best, sec = b - a, name
    return sec


def main():
    asm, sym, ksrc = sys.argv[1], sys.argv[2], sys.argv[3]
    hsrc = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(ksrc), "trace_dev.hpp")
    kname, hname = os.path.basename(ksrc), os.path.basename(hsrc)
    krng = kernel_ranges(Src(ksrc))
    hr = {hname: helper_ranges(Src(hsrc)), kname: helper_ranges(Src(ksrc))}
    counts = defaultdict(lambda: defaultdict(int))
    cur = "kernel prologue"
    inside = False
    depth = 0
    for line in open(asm):
        if not inside:
            inside = line.startswith(sym + ":")
            continue
        if line.startswith(".Lfunc_end"):
            break
        s = line.strip()
        if re.match(r"^(\.LBB\w+:|; %bb\.\d+:)", s):   # a block: its loop depth from the label comment
            m = re.search(r"Depth=(\d+)", line)
            depth = int(m.group(1)) if m else 0
            continue
        if s.startswith(".loc"):
            # the comment holds the inlining chain, innermost first: loc @[ caller @[ ... ] ]
            chain = re.findall(r"([\w./-]+):(\d+)(?::\d+)?", line.split(";", 1)[1]) if ";" in line else []
            chain = [(os.path.basename(f), int(l)) for f, l in chain if int(l) > 0]
            named = [innermost(hr[f], l, None) for f, l in chain if f in hr]
            named = [x for x in named if x]
            site = [l for f, l in chain if f == kname and innermost(krng, l, None)]
            if named:
                cur = named[-1]                  # the outermost helper that owns a section
            elif site:
                cur = innermost(krng, site[-1])  # the k_trace line the chain starts from
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        c = classify(s.split()[0])
        if c is None:
            continue
        sec = cur
        if sec.startswith("trav") and depth < 2:
            sec = "other"
        counts[sec][c] += 1
    cols = ["valu", "salu", "vmem", "smem", "lds", "scratch", "branch", "wait"]
    order = sorted(counts, key=lambda k: (not k.startswith("trav"), k))
    print("| section | " + " | ".join(cols) + " |")
    print("|---|" + "---|" * len(cols))
    tot = defaultdict(int)
    for k in order:
        for c in cols:
            tot[c] += counts[k][c]
        print(f"| {k} | " + " | ".join(str(counts[k][c]) for c in cols) + " |")
    print("| **total** | " + " | ".join(str(tot[c]) for c in cols) + " |")


if __name__ == "__main__":
    main()
