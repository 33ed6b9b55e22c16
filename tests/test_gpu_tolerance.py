"""GPU: the tolerance mode (TPT_FLAG_FAST; DESIGN.md section 4 "Tolerance mode")
against the oracle at every BASELINE configuration's full resolution.

The tolerance-mode build of the trace kernel contracts multiply-adds into FMAs,
runs the slab tests as one FMA per bound, and uses the hardware's approximate
reciprocal, square root, sine and cosine, without the culling guards; so its
image is not the reference's bit for bit, and SURVEY.md 8(d)'s per-channel
tolerance is the bar: mean |d| <= 1e-3, p99 |d| <= 1e-2, >= 99.5 % of pixels
within one 8-bit step of the oracle (test_gpu_parity.assert_parity with
bit_min=0).  The full-spp middle band of each configuration is checked in
tests/test_gpu_fullsize.py (mode "fast").  The exact mode stays the default.
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from oracle import oracle as O
from tests.conftest import scene_path
from tests.test_gpu_parity import assert_parity, image_metrics

pytestmark = pytest.mark.gpu

FULL = [
    # name, W, H, spp, depth, env
    ("box", 1920, 1080, 2, 8, None),
    ("ball", 1920, 1080, 2, 8, "sky"),
    ("tir", 1920, 1080, 2, 32, None),
    ("c5", 3840, 2160, 1, 8, None),
]


@pytest.mark.parametrize("name,W,H,spp,depth,env", FULL)
def test_tolerance_mode_full_resolution(name, W, H, spp, depth, env):
    s = T.Scene(scene_path(name))
    d = s.copySceneToDevice(0).build()
    try:
        sky = T.procedural_sky(2048, 1024) if env else None
        pt = T.PathTracer("", W, H, 0)
        if env:
            pt.envLight = T.EnvLight(sky, 0)
        rad = np.zeros((H, W, 3), np.float32)
        fb = np.zeros((H, W, 4), np.uint8)
        st = pt.doTrace(d, s.m_camera, fb, spp, seed=42, max_depth=depth, radiance=rad, flags=T._lib.FLAG_FAST)
        orad, obgra, oc = O.render(O.load_scene(scene_path(name)), W, H, spp, depth, 42,
                                   env=sky[::-1].copy() if env else None, trig_mode=1)
        m = image_metrics(rad, orad)
        print(name, "tolerance mode", m)
        assert_parity(m, bit_min=0.0)
        assert abs(st["traversals"] - oc["traversals"]) <= 0.01 * oc["traversals"]
        # the framebuffer is still copyToFB of the radiance
        q = np.clip(rad * 255.0, 0, 255).astype(np.uint8)[::-1]
        assert np.array_equal(fb[..., 0], q[..., 2]) and np.array_equal(fb[..., 2], q[..., 0])
    finally:
        d.close()


def test_tolerance_mode_discriminates():
    """The bar would catch a wrong image: another seed fails it."""
    s = T.Scene(scene_path("box"))
    d = s.copySceneToDevice(0).build()
    try:
        W, H, spp = 256, 144, 16
        pt = T.PathTracer("", W, H, 0)
        rad = np.zeros((H, W, 3), np.float32)
        pt.doTrace(d, s.m_camera, None, spp, seed=43, max_depth=8, radiance=rad, flags=T._lib.FLAG_FAST)
        orad, _, _ = O.render(O.load_scene(scene_path("box")), W, H, spp, 8, 42, trig_mode=1)
        m = image_metrics(rad, orad)
        assert m["mean"] > 1e-3 or m["within1"] < 0.995, m
    finally:
        d.close()


def test_exact_mode_is_the_default():
    s = T.Scene(scene_path("box"))
    d = s.copySceneToDevice(0).build()
    try:
        W, H, spp = 64, 36, 8
        pt = T.PathTracer("", W, H, 0)
        a = np.zeros((H, W, 3), np.float32)
        b = np.zeros((H, W, 3), np.float32)
        pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=8, radiance=a)
        pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=8, radiance=b, flags=T._lib.FLAG_FAST)
        orad, _, _ = O.render(O.load_scene(scene_path("box")), W, H, spp, 8, 42, trig_mode=1)
        assert np.array_equal(a.view(np.uint32), orad.view(np.uint32))
        assert not np.array_equal(b.view(np.uint32), orad.view(np.uint32))
    finally:
        d.close()
