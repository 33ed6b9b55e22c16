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
    print("golden fixtures written to", GOLD)
