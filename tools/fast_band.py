"""Tolerance mode (TPT_FLAG_FAST) against the oracle on a BASELINE configuration's
full-spp middle band (the band test_gpu_fullsize.py uses), with and without the
culling guards (TPT_FLAG_APPROX_CULL): SURVEY 8(d)'s image metrics per variant,
to separate rounding from different-triangle hits (verdict r05 item 1).
Usage: python tools/fast_band.py C5 [C2 ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinypathtracer_amd as T  # noqa: E402
from tests.conftest import scene_path  # noqa: E402
from tests.test_gpu_fullsize import ORACLE_BAND, _oracle_band  # noqa: E402
from tests.test_gpu_parity import image_metrics  # noqa: E402

VARIANTS = [("fast (guards kept)", T._lib.FLAG_FAST),
            ("fast + approx cull (no guards)", T._lib.FLAG_FAST | T._lib.FLAG_APPROX_CULL),
            ("exact", 0)]

for want in sys.argv[1:] or ["C5"]:
    cfg, name, W, H, spp, depth, env, env_is = next(c for c in ORACLE_BAND if c[0].replace(" ", "") == want)
    count = (H + 15) // 16
    band = (16, count, count // 2)
    s = T.Scene(scene_path(name))
    d = s.copySceneToDevice(0).build()
    sky = T.procedural_sky(2048, 1024) if env else None
    pt = T.PathTracer("", W, H, 0)
    if env:
        pt.envLight = T.EnvLight(sky, 0)
    orad, _, oc = _oracle_band(cfg, name, W, H, spp, depth, sky, env_is, band)
    rows = np.array([(y // 16) % count == band[2] for y in range(H)])
    for label, fl in VARIANTS:
        rad = np.zeros((H, W, 3), np.float32)
        st = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=rad, band=band,
                        flags=fl | (T._lib.FLAG_ENV_IS if env_is else 0))
        m = image_metrics(rad[rows], orad[rows])
        print(f"{cfg} band {band[2]} {spp} spp, {label}: mean {m['mean']:.3e} p99 {m['p99']:.4f} "
              f"within1 {m['within1']:.4f} bit {m['bit_same']:.4f} rays {st['traversals']} "
              f"(oracle {oc['traversals']}) trace {st['trace_ms']:.1f} ms", flush=True)
    d.close()
