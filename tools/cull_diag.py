"""Where does the culled ordered traversal (trace mode 1) differ from the
reference's visit order (mode 0)?  Diagnostic for tests/test_gpu_cull.py.

Prints, per scene, the divergence rate of
  * adversarial rays (tests/test_gpu_cull.adversarial_rays) split by origin kind
    (kernel hit point / triangle edge / vertex) and by the sine of the angle
    between the ray and the surface it leaves;
  * realistic rays: camera rays, then cosine-weighted bounces from their hit
    points (origin = o + t * d as the kernel computes it), several bounces deep;
and for the divergent rays the reference hit's conditioning (|cos| between the
ray and the hit triangle's normal, axis-aligned or not) and which side of the
cull (the reference's t below / above ours).
"""
import sys

import numpy as np

sys.path.insert(0, ".")
import tinypathtracer_amd as T  # noqa: E402
from tests.conftest import scene_path  # noqa: E402


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def tri_normals(wv, idx):
    tri = idx.reshape(-1, 3)
    v0, v1, v2 = wv[tri[:, 0]].astype(np.float64), wv[tri[:, 1]].astype(np.float64), wv[tri[:, 2]].astype(np.float64)
    n = np.cross(v1 - v0, v2 - v0)
    n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
    axis = (np.abs(n) > 1 - 1e-12).any(1)
    return n, axis, tri


def compare(d, o, dirs):
    h0, t0, uv0 = d.trace_rays(o, dirs, mode=0)
    h1, t1, uv1 = d.trace_rays(o, dirs, mode=1)
    bad = (h0 != h1) | (bits(t0) != bits(t1)) | (bits(uv0) != bits(uv1)).any(1)
    return bad, h0, t0, h1, t1


def realistic(d, s, n, depth, rng):
    wv, _ = d.read_world()
    nrm, _, tri = tri_normals(wv, s.indices)
    c2w = np.asarray(s.m_camera.c2w, np.float32).reshape(4, 4).T   # column-major
    org = np.tile(c2w[:3, 3], (n, 1)).astype(np.float32)
    th = np.tan(s.m_camera.vfov / 2)
    x = (rng.uniform(-1, 1, n) * th * s.m_camera.aspect)
    y = rng.uniform(-1, 1, n) * th
    dirs = (c2w[:3, :3] @ np.stack([x, y, -np.ones(n)]).astype(np.float32)).T.astype(np.float32)
    tot_bad, tot = 0, 0
    for _ in range(depth):
        bad, h0, t0, _, _ = compare(d, org, dirs)
        tot_bad += int(bad.sum())
        tot += len(org)
        ok = h0 >= 0
        if ok.sum() == 0:
            break
        org = (org[ok] + t0[ok][:, None] * dirs[ok]).astype(np.float32)
        nn = nrm[h0[ok]]
        k = len(org)
        # cosine-weighted hemisphere about the (flipped) geometric normal
        nn = np.where(((dirs[ok] * nn).sum(1) > 0)[:, None], -nn, nn)
        u1, u2 = rng.uniform(size=k), rng.uniform(size=k)
        a = np.where(np.abs(nn[:, 0:1]) > 0.5, np.array([[0, 1, 0]]), np.array([[1, 0, 0]]))
        b1 = np.cross(nn, a)
        b1 /= np.linalg.norm(b1, axis=1, keepdims=True)
        b2 = np.cross(nn, b1)
        r, phi = np.sqrt(u1), 2 * np.pi * u2
        dirs = (b1 * (r * np.cos(phi))[:, None] + b2 * (r * np.sin(phi))[:, None]
                + nn * np.sqrt(1 - u1)[:, None]).astype(np.float32)
    return tot_bad, tot


def main():
    from tests.test_gpu_cull import adversarial_rays
    names = sys.argv[1:] or ["box", "ball", "c5"]
    for name in names:
        s = T.Scene(scene_path(name))
        d = s.copySceneToDevice(0).build()
        d.scene_indices = s.indices
        wv, _ = d.read_world()
        nrm, axis, _ = tri_normals(wv, s.indices)
        rng = np.random.default_rng(1)
        o, dirs, kind, sin_a = adversarial_rays(d, 400_000, seed=3, kinds=True)
        bad, h0, t0, h1, t1 = compare(d, o, dirs)
        print(f"== {name}: adversarial {bad.sum()} / {len(o)} divergent")
        for k, lab in enumerate(("hit point", "edge", "vertex")):
            m = kind == k
            print(f"   origin {lab:9s}: {int(bad[m].sum())} / {int(m.sum())};  by sin(angle to surface):",
                  [(e, int(bad[m & (sin_a >= 10.0 ** e) & (sin_a < 10.0 ** (e + 1))].sum()))
                   for e in range(-8, 0)])
        idx = np.nonzero(bad)[0]
        if len(idx):
            hx = h0[idx]
            cos = np.abs((dirs[idx] / np.linalg.norm(dirs[idx], axis=1, keepdims=True) * nrm[np.maximum(hx, 0)]).sum(1))
            print("   ref miss", int((hx < 0).sum()), " ref hit axis-aligned", int(axis[hx[hx >= 0]].sum()),
                  " ref t < ours", int((t0[idx] < t1[idx]).sum()), " ref t > ours", int((t0[idx] > t1[idx]).sum()))
            print("   |cos(ray, ref hit normal)| quantiles", np.quantile(cos[hx >= 0], [0, 0.5, 0.9, 1.0]) if (hx >= 0).any() else "-")
            print("   ref t quantiles", np.quantile(t0[idx], [0, 0.25, 0.5, 0.75, 1.0]))
        for depth_rays in (2_000_000,):
            nb, nt = realistic(d, s, depth_rays, 6, rng)
            print(f"   realistic (camera + 5 cosine bounces): {nb} / {nt} divergent")
        d.close()




def dump(name="box2", out="gpurun_out/cull_examples.npz"):
    """Divergent adversarial rays with a well-conditioned reference hit."""
    from tests.test_gpu_cull import adversarial_rays
    s = T.Scene(scene_path(name))
    d = s.copySceneToDevice(0).build()
    d.scene_indices = s.indices
    wv, _ = d.read_world()
    nrm, _, _ = tri_normals(wv, s.indices)
    o, dirs, kind, sin_a = adversarial_rays(d, 400_000, seed=3, kinds=True)
    bad, h0, t0, h1, t1 = compare(d, o, dirs)
    idx = np.nonzero(bad)[0]
    np.savez(out, o=o[idx], d=dirs[idx], h0=h0[idx], t0=t0[idx], h1=h1[idx], t1=t1[idx], kind=kind[idx],
             sin_a=sin_a[idx], wv=wv)
    d.close()


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "dump":
        dump(*sys.argv[2:])
    else:
        main()
