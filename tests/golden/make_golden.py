"""Regenerate the committed golden fixtures (run in the build container).

  python tests/golden/make_golden.py

* images.npz: oracle renders (trig_mode 0 = libm float transcendentals, the
  semantics of the survey's host-compiled reference kernels, whose mean
  radiances SURVEY.md Appendix B records) for small configs, plus traversal
  counters -- pins the oracle against regressions;
* ref_l0_kat.json: outputs of the reference's OWN header-only math
  (include/math/*.h, transform.h via oracle/_ref/ref_kat) for every node
  transform in every shipped scene and a set of frsqrt / normalize / Mat4*Vec4
  inputs.  Needs /root/reference (build container only); the JSON travels.
* rng_kat.json: first 16 curand_uniform draws of the XORWOW restatement for
  seed 42 at subsequences {0, 1, 255, 65535, 2073599}.
"""
import json
import os
import struct
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
GOLD = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(GOLD, "scenes")

from oracle import oracle as O  # noqa: E402

IMAGE_CASES = [
    # key, scene, W, H, spp, depth
    ("box_64x36_s16_d8", "box", 64, 36, 16, 8),
    ("box_48x48_s16_d4", "box", 48, 48, 16, 4),
    ("box2_64x36_s16_d8", "box2", 64, 36, 16, 8),
    ("tir_64x36_s16_d32", "tir", 64, 36, 16, 32),
    ("ball_64x36_s16_d8", "ball", 64, 36, 16, 8),
    ("square_64x36_s16_d8", "square", 64, 36, 16, 8),
]


def hexf(x):
    return "%08x" % struct.unpack("<I", struct.pack("<f", float(x)))[0]


def make_images():
    out = {}
    meta = {}
    for key, name, W, H, spp, depth in IMAGE_CASES:
        ps = O.load_scene(os.path.join(SCENES, f"{name}.gltf"))
        rad, bgra, c = O.render(ps, W, H, spp, depth, 42, trig_mode=0)
        out[key + "_radiance"] = rad
        out[key + "_bgra"] = bgra
        meta[key] = {k: c[k] for k in ("traversals", "internal_visits", "leaf_tests", "shade_hits")}
    np.savez_compressed(os.path.join(GOLD, "images.npz"), **out)
    with open(os.path.join(GOLD, "images_meta.json"), "w") as f:
        json.dump(meta, f, indent=1)


def make_ref_kat():
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_kat")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_kat"])
    reqs, labels = [], []
    for fn in sorted(os.listdir(SCENES)):
        with open(os.path.join(SCENES, fn)) as f:
            model = json.load(f)
        for ni, node in enumerate(model.get("nodes", [])):
            r = node.get("rotation")
            q = (r[0], r[1], r[2], r[3]) if r else (0.0, 0.0, 0.0, 0.0)
            s = node.get("scale", [1.0, 1.0, 1.0])
            t = node.get("translation", [0.0, 0.0, 0.0])
            vals = [t[0], t[1], t[2], q[0], q[1], q[2], q[3], s[0], s[1], s[2]]
            reqs.append("T " + " ".join(hexf(np.float32(v)) for v in vals))
            labels.append({"scene": fn, "node": ni, "in": [hexf(np.float32(v)) for v in vals]})
    rng = np.random.default_rng(5)
    for x in list(rng.uniform(1e-4, 100.0, 24).astype(np.float32)) + [np.float32(1.0), np.float32(0.25)]:
        reqs.append("R " + hexf(x))
        labels.append({"frsqrt": hexf(x)})
    for v in rng.normal(size=(24, 3)).astype(np.float32):
        reqs.append("N " + " ".join(hexf(c) for c in v))
        labels.append({"normalize": [hexf(c) for c in v]})
    for _ in range(12):
        m = rng.normal(size=16).astype(np.float32)
        v = rng.normal(size=4).astype(np.float32)
        reqs.append("V " + " ".join(hexf(c) for c in list(m) + list(v)))
        labels.append({"matvec": [hexf(c) for c in list(m) + list(v)]})
    res = subprocess.run([exe], input="\n".join(reqs) + "\n", capture_output=True, text=True, check=True)
    lines = res.stdout.strip().split("\n")
    assert len(lines) == len(reqs)
    kat = []
    for lab, line in zip(labels, lines):
        parts = line.split()
        lab["out"] = parts[1:]
        kat.append(lab)
    with open(os.path.join(GOLD, "ref_l0_kat.json"), "w") as f:
        json.dump({"source": "reference include/math/{vec,mat,quat}.h, transform.h via oracle/_ref/ref_kat",
                   "kat": kat}, f, indent=0)


def hot_kat_cases():
    """Inputs for the reference's header-only hot-path functions (float32):
    rayHitBBox, rayHitTriangle, DeltaLight::sample, CalcDistAttenuation,
    Spectrum::toUChar, Material().  Random cases plus the edge cases the
    traversal meets: zero / signed-zero / denormal / infinite / NaN direction
    components, origins on slab planes, flat and inverted boxes, rays parallel
    to a triangle's plane (denom == 0), u + v == 1 edges, negative and
    near-Delta distances, grazing rays, lights at the shading point and beyond
    the attenuation radius, bytes at and beyond [0, 1]."""
    f32 = np.float32
    rng = np.random.default_rng(20260)
    inf, nan = np.inf, np.nan
    box = []
    for _ in range(400):
        o = rng.normal(0, 3, 3)
        d = rng.normal(0, 1, 3)
        a, b = rng.normal(0, 2, 3), rng.normal(0, 2, 3)
        box.append(list(o) + list(d) + list(np.minimum(a, b)) + list(np.maximum(a, b)))
    special_d = [0.0, -0.0, 1e-45, -1e-45, 1e-40, inf, -inf, nan, 1.0, -1.0, 3.0e38]
    special_o = [-1.0, 0.0, 0.5, 1.0, 2.0, -0.0, inf, -inf, nan]
    for _ in range(500):
        o = [rng.choice(special_o) if rng.random() < 0.5 else rng.normal(0, 2) for _ in range(3)]
        d = [rng.choice(special_d) if rng.random() < 0.5 else rng.normal(0, 1) for _ in range(3)]
        lo = np.array([0.0, 0.0, 0.0])
        hi = np.array([1.0, 1.0, 1.0])
        k = rng.integers(6)
        if k == 1:      # flat box
            hi[rng.integers(3)] = 0.0
        elif k == 2:    # point box
            hi = lo.copy()
        elif k == 3:    # BBox() default: (REAL_MAX, -REAL_MAX)
            lo[:] = 3.4028234663852886e38
            hi[:] = -3.4028234663852886e38
        elif k == 4:    # box behind the origin
            lo -= 10.0
            hi -= 10.0
        box.append(list(o) + list(d) + list(lo) + list(hi))
    tri = []
    for _ in range(400):
        v = rng.normal(0, 1, 9)
        c = (v[0:3] + v[3:6] + v[6:9]) / 3.0
        o = rng.normal(0, 3, 3)
        d = c + rng.normal(0, 0.5, 3) - o
        tri.append(list(o) + list(d) + list(v))
    T0 = [0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0, 0.0]   # unit right triangle in z = 0
    for o, d in [((0.25, 0.25, 1.0), (0.0, 0.0, -1.0)),      # inside
                 ((0.5, 0.5, 1.0), (0.0, 0.0, -1.0)),        # u + v == 1 edge
                 ((0.0, 0.0, 1.0), (0.0, 0.0, -1.0)),        # vertex v0
                 ((1.0, 0.0, 1.0), (0.0, 0.0, -1.0)),        # vertex v1
                 ((0.0, 0.5, 1.0), (0.0, 0.0, -1.0)),        # u == 0 edge
                 ((0.5, 0.0, 1.0), (0.0, 0.0, -1.0)),        # v == 0 edge
                 ((0.6, 0.5, 1.0), (0.0, 0.0, -1.0)),        # just outside u + v = 1
                 ((0.25, 0.25, 1.0), (0.0, 0.0, 1.0)),       # negative t
                 ((0.25, 0.25, -1.0), (0.0, 0.0, 1.0)),      # from below
                 ((0.25, 0.25, 2e-4), (0.0, 0.0, -1.0)),     # t == Delta
                 ((0.25, 0.25, 1e-4), (0.0, 0.0, -1.0)),     # t below Delta
                 ((0.25, 0.25, 0.0), (0.0, 0.0, -1.0)),      # origin on the plane
                 ((-1.0, 0.25, 0.0), (1.0, 0.0, 0.0)),       # parallel, in plane: denom == 0
                 ((-1.0, 0.25, 1.0), (1.0, 0.5, 0.0)),       # parallel, above
                 ((-1.0, 0.25, 1e-3), (1.0, 0.0, -1e-3)),    # grazing
                 ((-1.0, 0.25, 1e-6), (1.0, 0.0, -1e-6)),    # grazing, tiny slope
                 ((0.25, 0.25, 1.0), (0.0, 0.0, 0.0)),       # zero direction
                 ((0.25, 0.25, 1.0), (0.0, 0.0, -inf)),
                 ((0.25, 0.25, 1.0), (nan, 0.0, -1.0)),
                 ((0.25, 0.25, inf), (0.0, 0.0, -1.0))]:
        tri.append(list(o) + list(d) + T0)
    for o, d in [((0.25, 0.25, 1.0), (0.0, 0.0, -1.0))] * 2:
        tri.append(list(o) + list(d) + [0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 1.0, 1.0, 0.0])   # v1 == v0
        tri.append(list(o) + list(d) + [0.0, 0.0, 0.0, 1.0, 1.0, 0.0, 2.0, 2.0, 0.0])   # collinear
    for _ in range(200):   # secondary rays leaving a surface near a corner: t near Delta, grazing
        v = rng.normal(0, 1, 9)
        w = rng.dirichlet([1.0, 1.0, 1.0])
        p = w[0] * v[0:3] + w[1] * v[3:6] + w[2] * v[6:9]
        n = np.cross(v[3:6] - v[0:3], v[6:9] - v[0:3])
        n /= np.linalg.norm(n)
        dd = rng.normal(0, 1, 3)
        dd -= np.dot(dd, n) * n * (1.0 - 10.0 ** rng.uniform(-6, 0))
        o = p - dd * 10.0 ** rng.uniform(-5, -2)
        tri.append(list(o) + list(dd) + list(v))
    light = []
    for _ in range(120):
        t = int(rng.integers(3))
        col = list(rng.uniform(0, 1, 3))
        inten = float(rng.uniform(0.1, 5.0))
        pos = list(rng.normal(0, 4, 3))
        dd = rng.normal(0, 1, 3)
        dd /= np.linalg.norm(dd)
        co = float(np.cos(rng.uniform(0.1, 1.2)))
        inv = float(1.0 / max(np.cos(rng.uniform(0.0, 0.1)) - co, 1e-3))
        p = list(rng.normal(0, 4, 3) * (3.0 if rng.random() < 0.2 else 1.0))
        light.append([t] + col + [inten] + pos + list(dd) + [co, inv] + p)
    for t in (0, 2):
        light.append([t, 1.0, 1.0, 1.0, 2.0, 1.0, 2.0, 3.0, 0.0, -1.0, 0.0, 0.5, 2.0, 1.0, 2.0, 3.0])  # p == pos
        light.append([t, 1.0, 0.5, 0.25, 2.0, 0.0, 0.0, 0.0, 0.0, -1.0, 0.0, 0.5, 2.0, 0.0, -10.0, 0.0])  # d == 10
        light.append([t, 1.0, 0.5, 0.25, 2.0, 0.0, 0.0, 0.0, 0.0, -1.0, 0.0, 0.5, 2.0, 0.0, -3.0, 0.0])
    att = [[x, 1.0, 0.5, 0.25] for x in (0.0, -0.0, 1.0, 3.0, 9.99, 10.0, 10.01, 100.0, 1e20, inf, nan, 1e-30)]
    att += [[float(x), 1.0, 2.0, 3.0] for x in rng.uniform(0, 12, 40)]
    uch = [[-1.0, -0.0, 0.0], [1.0 / 255, 0.5 / 255, 0.999], [1.0, 1.5, 255.5 / 255], [inf, -inf, nan],
           [1e-45, 0.99999994, 1.0000001], [254.5 / 255, 253.99 / 255, 2.0], [-1e-30, 1e30, 0.5]]
    uch += [list(x) for x in rng.uniform(-0.2, 1.2, (60, 3))]
    cast = lambda rows: [[f32(x) for x in r] for r in rows]
    return {"B": cast(box), "X": cast(tri), "L": cast(light), "A": cast(att), "U": cast(uch)}


def make_ref_hot_kat():
    """tests/golden/ref_hot_kat.json: the reference's own geometry_queries.h,
    delta_light.h and material.h, compiled by hipcc (host only) from
    /root/reference/include (oracle/_ref/ref_hot_kat), on hot_kat_cases()."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_hot_kat")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "_ref/ref_hot_kat"])
    cases = hot_kat_cases()
    reqs, keys = [], []
    for op, rows in cases.items():
        for r in rows:
            if op == "L":   # light type is an integer token
                reqs.append("L %d " % int(r[0]) + " ".join(hexf(x) for x in r[1:]))
            else:
                reqs.append(op + " " + " ".join(hexf(x) for x in r))
            keys.append(op)
    reqs.append("M")
    keys.append("M")
    reqs.append("S")
    keys.append("S")
    res = subprocess.run([exe], input="\n".join(reqs) + "\n", capture_output=True, text=True, check=True)
    lines = res.stdout.strip().split("\n")
    assert len(lines) == len(reqs)
    out = {k: [] for k in ("B", "X", "L", "A", "U", "M", "S")}
    for op, req, line in zip(keys, reqs, lines):
        parts = line.split()
        assert parts[0] == op, (req, line)
        out[op].append({"in": req.split()[1:], "out": parts[1:]})
    with open(os.path.join(GOLD, "ref_hot_kat.json"), "w") as f:
        json.dump({"source": "reference include/geometry_queries.h:18-86, delta_light.h:25-130, "
                             "material.h:74-103 via oracle/_ref/ref_hot_kat (hipcc --cuda-host-only)",
                   "protocol": "oracle/ref_hot_kat.cpp header", "kat": out}, f, indent=0)


def make_rng_kat():
    kat = {}
    for sub in (0, 1, 255, 65535, 2073599):
        kat[str(sub)] = [hexf(u) for u in O.uniform_stream(42, sub, 16)]
    with open(os.path.join(GOLD, "rng_kat.json"), "w") as f:
        json.dump({"seed": 42, "uniforms": kat}, f, indent=1)


if __name__ == "__main__":
    make_images()
    make_rng_kat()
    if os.path.isdir("/root/reference/include"):
        make_ref_kat()
        make_ref_hot_kat()
    print("golden fixtures written to", GOLD)
