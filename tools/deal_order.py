"""One rank's share of an N-way C5 split rendered with its bands in different
orders (tpt_params.band_list; every order is the same pixels, bit-identical):
ms per frame per order.  Usage: python tools/deal_order.py [N] [ranks...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinypathtracer_amd as T  # noqa: E402
from tests.conftest import scene_path  # noqa: E402
from tinypathtracer_amd import shard  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
ranks = [int(v) for v in sys.argv[2:]] or [7, 0]
W, H, spp = 3840, 2160, 2048
s = T.Scene(scene_path("c5"))
d = s.copySceneToDevice(0).build()
pt = T.PathTracer("", W, H, 0)
nb = shard.n_bands(H, 16)


def frame(lst):
    d.build(asynchronous=True)
    t = time.perf_counter()
    st = pt.doTrace(d, s.m_camera, None, spp, seed=42, band=(16, N, 0), band_list=lst)
    return (time.perf_counter() - t) * 1e3, st


for r in ranks:
    base = list(range(r, nb, N))
    orders = {"ascending": base, "descending": base[::-1], "rotated-half": base[len(base) // 2:] + base[:len(base) // 2],
              "outside-in": [b for p in zip(base[: (len(base) + 1) // 2], base[::-1][: len(base) // 2]) for b in p]
              + ([base[len(base) // 2]] if len(base) % 2 else [])}
    frame(base)   # warm-up
    for name, lst in orders.items():
        assert sorted(lst) == base
        ms = [frame(lst)[0] for _ in range(2)]
        print(f"rank {r} of {N} ({len(base)} bands) {name}: {min(ms):.1f} ms ({ms[0]:.1f}, {ms[1]:.1f})", flush=True)
d.close()
