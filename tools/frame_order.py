"""A whole frame (N = 1) rendered with its bands in different dispatch orders
(tpt_params.band_list; the same pixels, bit-identical): ms per frame per
order, interleaved reps.  Usage: python tools/frame_order.py C2|C5 [reps]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinypathtracer_amd as T  # noqa: E402
from tests.conftest import scene_path  # noqa: E402
from tinypathtracer_amd import shard  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
name, W, H, spp = {"C2": ("box", 1920, 1080, 1024), "C5": ("c5", 3840, 2160, 512)}[cfg]
s = T.Scene(scene_path(name))
d = s.copySceneToDevice(0).build()
pt = T.PathTracer("", W, H, 0)
nb = shard.n_bands(H, 16)
short = nb - 1 if H % 16 else None
base = list(range(nb))
full = [b for b in base if b != short]
mid = len(full) // 2


def fix(lst):   # the short band last
    return [b for b in lst if b != short] + ([short] if short is not None else [])


orders = {
    "natural": None,
    "ascending-list": base,
    "descending": fix(base[::-1]),
    "outside-in": fix([b for p in zip(full[: (len(full) + 1) // 2], full[::-1][: len(full) // 2]) for b in p]
                      + ([full[mid]] if len(full) % 2 else [])),
    "middle-out": fix(sorted(full, key=lambda b: (abs(b - mid), b))),
    "rotated-half": fix(full[mid:] + full[:mid]),
}
ref = None
for rep in range(reps + 1):
    for k, lst in orders.items():
        d.build(asynchronous=True)
        rad = np.zeros((H, W, 3), np.float32) if rep == 0 else None
        t = time.perf_counter()
        st = pt.doTrace(d, s.m_camera, None, spp, seed=42, band_list=lst, radiance=rad)
        ms = (time.perf_counter() - t) * 1e3
        if rep == 0:   # warm-up: every order renders the same frame
            if ref is None:
                ref = rad
            assert np.array_equal(rad.view(np.uint32), ref.view(np.uint32)), k
            continue
        print(f"{cfg} rep {rep} {k}: {ms:.1f} ms, {st['traversals'] / ms / 1e3:.0f} Mrays/s", flush=True)
d.close()
