"""Lone-wave per-step latency of the traversal (verdict r04 item 1; DESIGN.md section 6,
"The drained chain").  tpt_debug_step_latency runs ONE 64-lane wave over up to 64
closest-hit rays; this script feeds it the strong-scaled C2 chain's kind of ray --
chords through box.gltf's glass sphere, from a point on one of its triangles to
another (the refracted rays the heavy pixels' samples chain) -- and camera rays for
comparison, with the 4-wide nodes in global memory (as k_trace reads them) or the
whole main tree in LDS, in exact and tolerance mode.  Prints shader cycles per loop
iteration of the wave and per visit of its busiest lane (best of 5 runs each).
Usage (GPU): python tools/step_latency.py [scene]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinypathtracer_amd as T  # noqa: E402
from tests.conftest import scene_path  # noqa: E402


def rays(scene, d, kind, n, rng):
    wv, _ = d.read_world()
    idx = scene.indices.reshape(-1, 3)
    cen = wv[idx].mean(axis=1)
    if kind == "camera":
        org = np.tile(scene.m_camera.c2w.reshape(4, 4)[3, :3], (n, 1))
        tgt = cen[rng.integers(0, len(cen), n)]
        return org.astype(np.float32), (tgt - org).astype(np.float32)
    # the glass sphere: faces of the dielectric material (eta > 0)
    mat_of_face = np.zeros(len(idx), np.int32)
    lut = scene.lut
    for o in range(len(lut)):
        end = lut[o + 1][0] if o + 1 < len(lut) else len(idx)
        mat_of_face[lut[o][0]:end] = lut[o][1]
    eta = scene.materials[:, 4] if len(scene.materials) else np.zeros(1)
    glass = np.nonzero(eta[np.clip(mat_of_face, 0, len(eta) - 1)] > 0)[0]
    a = glass[rng.integers(0, len(glass), n)]
    b = glass[rng.integers(0, len(glass), n)]
    org, tgt = cen[a], cen[b]
    return org.astype(np.float32), (tgt - org).astype(np.float32)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "box"
    s = T.Scene(scene_path(name))
    d = s.copySceneToDevice(0).build()
    rng = np.random.default_rng(5)
    out = {}
    for kind in ("glass chords", "camera"):
        for nr in (64, 8, 1):
            o, dr = rays(s, d, kind, nr, rng)
            for mode, mname in ((0, "global"), (1, "lds")):
                for flags, fname in ((0, "exact"), (T._lib.FLAG_FAST, "fast")):
                    best = None
                    try:
                        for _ in range(5):
                            steps, iters, cyc, fid = d.step_latency(o, dr, mode, flags)
                            if best is None or cyc < best[2]:
                                best = (steps, iters, cyc)
                    except T.TPTError as e:
                        print(kind, nr, mname, fname, "skipped:", e)
                        continue
                    steps, iters, cyc = best
                    key = f"{kind} x{nr} nodes={mname} {fname}"
                    out[key] = {"cycles": cyc, "wave_iterations": iters, "max_lane_steps": int(steps.max()),
                                "mean_lane_steps": round(float(steps.mean()), 2),
                                "cycles_per_iteration": round(cyc / max(iters, 1), 1)}
                    print(f"{key:45s} iterations {iters:5d}  busiest lane {int(steps.max()):4d} steps  "
                          f"mean {steps.mean():6.2f}  cycles/iteration {cyc / max(iters, 1):7.1f}")
    # four lanes per ray (mode 2) against one lane per ray on the same rays: the
    # wave's whole walk in cycles (the chain latency of its slowest ray) and the hits
    quad = {}
    for kind in ("glass chords", "camera"):
        for nr in (16, 4, 1):
            # (the four-lane walk takes finite rays only; a direction with a zero
            # component has an infinite 1/d and takes the binary path in the render)
            o, dr = rays(s, d, kind, 8 * nr, rng)
            keep = np.nonzero(np.all(dr != 0.0, axis=1))[0][:nr]
            o, dr = o[keep], dr[keep]
            res = {}
            for mode, mname in ((0, "one lane"), (2, "four lanes")):
                best = None
                for _ in range(5):
                    steps, iters, cyc, fid = d.step_latency(o, dr, mode, 0)
                    if best is None or cyc < best[2]:
                        best = (steps, iters, cyc, fid)
                res[mname] = best
            same = bool(np.array_equal(res["one lane"][3], res["four lanes"][3]))
            if not same:
                bad = np.nonzero(res["one lane"][3] != res["four lanes"][3])[0]
                hit0, _, _ = d.trace_rays(o[bad], dr[bad], mode=0)
                hit1, _, _ = d.trace_rays(o[bad], dr[bad], mode=1)
                print("  differing rays", bad.tolist(), "one lane", res["one lane"][3][bad].tolist(), "four lanes",
                      res["four lanes"][3][bad].tolist(), "reference order", np.asarray(hit0).tolist(),
                      "render", np.asarray(hit1).tolist())
            c1, c4 = res["one lane"][2], res["four lanes"][2]
            key = f"{kind} x{nr}"
            quad[key] = {"one_lane_cycles": c1, "four_lane_cycles": c4, "ratio": round(c4 / max(c1, 1), 3),
                         "one_lane_busiest_steps": int(res["one lane"][0].max()),
                         "four_lane_busiest_visits": int(res["four lanes"][0].max()),
                         "one_lane_iterations": res["one lane"][1], "four_lane_iterations": res["four lanes"][1],
                         "same_hits": same}
            print(f"{key:22s} one lane {c1:7d} cycles ({res['one lane'][1]:4d} iterations)  four lanes {c4:7d} "
                  f"({res['four lanes'][1]:4d} iterations)  ratio {c4 / max(c1, 1):.3f}  same hits {same}")
    print(json.dumps({"scene": name, "results": out, "four_lanes": quad}))
    d.close()


if __name__ == "__main__":
    main()
