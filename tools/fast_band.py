"""Tolerance-mode variants on C5's full-spp middle band against the oracle's band
(scratch_oracle/c5_band.npz, computed on the CPU by the same oracle render the
test uses): the SURVEY 8(d) image metrics.  Usage: TPT_LIB=... python tools/fast_band.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tinypathtracer_amd as T  # noqa: E402
from tests.conftest import scene_path  # noqa: E402
from tests.test_gpu_parity import image_metrics  # noqa: E402

z = np.load(os.path.join(ROOT, "scratch_oracle", "c5_band.npz"))
W, H, spp = 3840, 2160, 2048
count = (H + 15) // 16
band = (16, count, count // 2)
s = T.Scene(scene_path("c5"))
d = s.copySceneToDevice(0).build()
pt = T.PathTracer("", W, H, 0)
rad = np.zeros((H, W, 3), np.float32)
st = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=8, radiance=rad, band=band, flags=T._lib.FLAG_FAST)
m = image_metrics(rad[z["rows"]], z["rad"])
print(os.environ.get("TPT_LIB", "libtpt.so").split("/")[-2], "C5 band fast:", m, "rays", st["traversals"],
      "oracle", int(z["traversals"]))
