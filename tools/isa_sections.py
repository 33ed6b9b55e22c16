#!/usr/bin/env python3
"""Static instruction counts of one k_trace variant by source section
("ISA breakdown").

usage: isa_sections.py dump_g.s KERNEL_SYMBOL trace.hip

dump_g.s: a `hipcc -O3 -g --cuda-device-only -S` dump of trace.hip; the
kernel is read from its label to the next .Lfunc_end.  Every instruction is charged to the
trace.hip line of its .loc; instructions of inlined helpers in other files
(tpt_math.hpp, ptrig.hpp, rng.hpp) are charged to the last trace.hip line
before them (their call site).  trace.hip lines map to sections through the
function / marker ranges found in the source itself, so the table follows the
code as it moves.  Counts are static (code size per section); per-visit
costs follow because a wave runs a section's straight-line code once per
iteration in which any lane takes it.
"""
import re
import sys
from collections import OrderedDict, defaultdict


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


def section_map(src):
    """[(first_line, last_line, section)] from the source text."""
    lines = open(src).read().split("\n")

    def find(pat, start=0):
        for i in range(start, len(lines)):
            if re.search(pat, lines[i]):
                return i + 1
        raise SystemExit(f"pattern not found: {pat}")

    def func(name):   # a function's line range: its signature to the closing brace at column 0
        a = find(r"__forceinline__ .*\b" + name + r"\(")
        b = a
        while not lines[b - 1].startswith("}"):
            b += 1
        return a, b

    rng = []
    for name, sec in [("box_hit", "trav: binary visit"), ("inner_visit", "trav: binary visit"),
                      ("slab_minmax", "trav: 4-wide visit"), ("inner_visit4", "trav: 4-wide visit"),
                      ("tri_core", "trav: leaf test"), ("cull_slack", "trav: leaf test"),
                      ("leaf_test_q", "trav: leaf test"), ("leaf_test", "trav: leaf test"),
                      ("sliver_scan", "pass: sliver re-test"), ("sliver_pass", "pass: sliver re-test"),
                      ("new_direction", "pass: BSDF sample (getNewDirection)"),
                      ("probe_misses_emitters", "pass: probe pre-test"),
                      ("trav_begin", "pass: ray set-up (trav_begin)"), ("grazing", "pass: grazing test"),
                      ("light_sample", "pass: delta lights"), ("env_lookup_inl", "pass: env lookup"),
                      ("env_is_sample", "pass: env IS"), ("emit_probe_inline", "pass: inline emitter test")]:
        try:
            a, b = func(name)
        except SystemExit:   # (older sources: a helper that does not exist)
            continue
        rng.append((a, b, sec))
    # helpers charged to their caller's section (records, stack, RNG glue)
    for pat, sec in [(r"^struct PathRecords", "helper"), (r"^struct LaneStack", "helper")]:
        a = find(pat)
        b = a
        while not lines[b - 1].startswith("};"):
            b += 1
        rng.append((a, b, sec))
    for name in ("stack_slot_offset", "p_kind", "lds_f4", "band_row", "wave_sum", "fsincos_2pi"):
        try:
            a, b = func(name)
            rng.append((a, b, "helper"))
        except SystemExit:
            pass
    k = find(r"^void k_trace\(")
    loop_top = find(r"^    for \(;;\) \{", k)
    done = find(r"if \(ts == TS_DONE\) \{", loop_top + 1)
    s1 = find(r"TPT_SEC\(1\)", done)
    s2 = find(r"TPT_SEC\(2\)", s1)
    s3 = find(r"TPT_SEC\(3\)", s2)
    s4 = find(r"TPT_SEC\(4\)", s3)
    s5 = find(r"TPT_SEC\(5\)", s4)
    s6 = find(r"TPT_SEC\(6\)", s5)
    tl = find(r"const int thr = refill;", s6)
    leafdec = find(r"const unsigned long long hb = __ballot\(has\);", tl)
    tend = find(r"if \(ts == TS_TRAV && r.node < 0 && r.pend < 0\) ts = TS_DONE;", leafdec)
    kend = find(r"^}", tend)
    rng += [(k, loop_top, "kernel prologue"), (loop_top, done, "pass: sliver / probe pass-2 hand-over"),
            (done, s1, "pass: consume (hit prelude, env miss)"), (s1, s2, "pass: lights / probe set-up"),
            (s2, s3, "pass: after (next bounce)"), (s3, s4, "pass: unwind"), (s4, s5, "pass: camera ray"),
            (s5, s6, "pass: ray set-up (trav_begin)"), (s6, tl, "pass: exit test"),
            (tl, leafdec, "trav: loop control, stack pop, leaf park"),
            (leafdec, tend, "trav: leaf-test decision"), (tend, tend + 2, "trav: loop control, stack pop, leaf park"),
            (tend + 3, kend, "kernel epilogue (state write-back, counters)")]
    return rng, (tend, kend)


def main():
    asm, sym, src = sys.argv[1], sys.argv[2], sys.argv[3]
    srcname = src.split("/")[-1]
    rng, _ = section_map(src)
    files = {}
    for line in open(asm):
        m = re.match(r"\s*\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", line)
        if m:
            files[m.group(1)] = m.group(2)
    counts = defaultdict(lambda: defaultdict(int))
    def section_of(ln):   # the innermost range holding line ln
        sec, best = "other", None
        for a, b, name in rng:
            if a <= ln <= b and (best is None or b - a < best):
                best, sec = b - a, name
        return sec

    cur_file, cur_line, last_main = None, 0, 0
    cur_sec = ["kernel prologue"]
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
            p = s.split()
            cur_file, cur_line = files.get(p[1], p[1]), int(p[2])
            # the comment holds the inlining chain: loc @[ caller @[ caller's caller ] ]
            chain = re.findall(r"([\w./-]+):(\d+)(?::\d+)?", line.split(";", 1)[1]) if ";" in line else []
            main = [int(l) for f, l in chain if f.endswith(srcname) and int(l) > 0]
            if main:
                # the outermost function below k_trace that owns a section decides
                # (slab_minmax inside probe_misses_emitters is the probe pre-test);
                # otherwise the k_trace call-site line does
                site = main[-1]
                named = [section_of(l) for l in main[:-1]]
                named = [x for x in named if x not in ("helper", "other") and not x.startswith(("kernel", "pass: consume",
                         "pass: lights", "pass: after", "pass: unwind", "pass: camera", "pass: exit", "pass: sliver /"))]
                sec = named[-1] if named else section_of(site)
                if sec == "helper":
                    sec = section_of(site)
                last_main = site
                cur_sec[0] = sec
            continue
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        c = classify(s.split()[0])
        if c is None:
            continue
        sec = cur_sec[0]
        if sec == "helper" or (sec.startswith("trav") and depth < 2):
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
