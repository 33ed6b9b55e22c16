"""GPU parity of four lanes per pixel (tpt_params.lanes_per_pixel = 4, k_trace QUAD;
DESIGN.md section 6, "Four lanes per ray").

Every lane of a quad runs the pixel's path (the reference's per-pixel loops,
path_tracer.cu:296-435) with the same state; each 4-wide node visit is split over
the four lanes (child k on lane k, leaf children tested at once, the best hit kept
under the ordered tie rule).  The closest hit does not depend on the visit order,
so the frame must be the one-lane kernel's bit for bit, with the same ray counts,
and the oracle's.
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from oracle import oracle as O
from tests.conftest import scene_path
from tests.test_gpu_parity import CASES, assert_parity, image_metrics

pytestmark = pytest.mark.gpu

# scenes without delta lights (the QUAD variants run the one-lane logic)
QUAD_CASES = [c for c in CASES if c[0] not in ("ball", "square")]
SCENES = sorted({c[0] for c in QUAD_CASES})
STATS = ("traversals", "local_rays", "shade_hits", "pixels", "samples")


@pytest.fixture(scope="module")
def built():
    out = {}
    for name in SCENES + ["ball"]:
        s = T.Scene(scene_path(name))
        out[name] = (s, s.copySceneToDevice(0).build(), O.load_scene(scene_path(name)))
    yield out
    for _, d, _ in out.values():
        d.close()


def _render(s, d, W, H, spp, depth, env, lanes, seed=42, **kw):
    pt = T.PathTracer("", W, H, 0)
    if env is not None:
        pt.envLight = T.EnvLight(env, 0)
    rad = np.zeros((H, W, 3), np.float32)
    fb = np.zeros((H, W, 4), np.uint8)
    st = pt.doTrace(d, s.m_camera, fb, spp, seed=seed, max_depth=depth, radiance=rad, lanes_per_pixel=lanes, **kw)
    return rad, fb, st


def _same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("name,W,H,spp,depth,env", QUAD_CASES)
def test_quad_matches_one_lane_and_oracle(built, name, W, H, spp, depth, env):
    s, d, o = built[name]
    sky = T.procedural_sky(64, 32) if env else None
    rad1, fb1, st1 = _render(s, d, W, H, spp, depth, sky, 1)
    rad4, fb4, st4 = _render(s, d, W, H, spp, depth, sky, 4)
    assert _same(rad4, rad1)
    assert np.array_equal(fb4, fb1)
    for k in STATS:
        assert st4[k] == st1[k], k
    orad, obgra, oc = O.render(o, W, H, spp, depth, 42, env=sky[::-1].copy() if env else None, trig_mode=1)
    assert_parity(image_metrics(rad4, orad))
    assert np.array_equal(fb4[..., :3], obgra[..., :3])
    assert st4["traversals"] == oc["traversals"]


def test_quad_bands_frames_progressive_and_tolerance_mode(built):
    s, d, o = built["box"]
    W, H, spp = 64, 48, 8
    full, _, _ = _render(s, d, W, H, spp, 8, None, 4)
    one, _, _ = _render(s, d, W, H, spp, 8, None, 1)
    assert _same(full, one)
    acc = np.zeros_like(full)   # interleaved 16-row bands (the strong-scaled split)
    for b in range(3):
        part, _, _ = _render(s, d, W, H, spp, 8, None, 4, band=(16, 3, b))
        rows = [y for y in range(H) if (y // 16) % 3 == b]
        acc[rows] = part[rows]
    assert _same(acc, full)
    pt = T.PathTracer("", W, H, 0)   # progressive: 4 + 4 spp == 8 spp
    r1 = np.zeros((H, W, 3), np.float32)
    pt.doTrace(d, s.m_camera, None, 4, seed=42, max_depth=8, radiance=r1, lanes_per_pixel=4)
    pt.doTrace(d, s.m_camera, None, 4, seed=42, max_depth=8, radiance=r1, lanes_per_pixel=4, accumulate=True)
    assert _same(r1, full)
    pt = T.PathTracer("", W, H, 0)   # a batch of frames
    rads = [np.zeros((H, W, 3), np.float32) for _ in range(2)]
    pt.doTraceFrames(d, s.m_camera, [42, 43], None, spp, max_depth=8, radiances=rads, lanes_per_pixel=4)
    one43, _, _ = _render(s, d, W, H, spp, 8, None, 1, seed=43)
    assert _same(rads[0], full)
    assert _same(rads[1], one43)
    fast4, _, _ = _render(s, d, W, H, spp, 8, None, 4, flags=T._lib.FLAG_FAST)   # tolerance build: same hits too
    fast1, _, _ = _render(s, d, W, H, spp, 8, None, 1, flags=T._lib.FLAG_FAST)
    assert _same(fast4, fast1)


def test_quad_refused_where_the_one_lane_logic_does_not_apply(built):
    s, d, o = built["ball"]   # a point light: pair-mode logic
    with pytest.raises(T.TPTError):
        _render(s, d, 32, 16, 2, 8, T.procedural_sky(64, 32), 4)
    s, d, o = built["box"]
    with pytest.raises(T.TPTError):
        _render(s, d, 32, 16, 2, 8, None, 4, flags=T._lib.FLAG_REF_ORDER)
    with pytest.raises(T.TPTError):
        _render(s, d, 32, 16, 2, 8, None, 3)


@pytest.mark.parametrize("name,W,H,spp,depth", [
    ("box", 1920, 1080, 4, 8),
    ("tir", 1920, 1080, 4, 32),
    ("c5", 3840, 2160, 1, 8),
])
def test_quad_full_resolution_equals_one_lane(built, name, W, H, spp, depth):
    s, d, o = built[name]
    rad1, fb1, st1 = _render(s, d, W, H, spp, depth, None, 1)
    rad4, fb4, st4 = _render(s, d, W, H, spp, depth, None, 4)
    assert _same(rad4, rad1)
    assert np.array_equal(fb4, fb1)
    for k in STATS:
        assert st4[k] == st1[k], k


def test_quad_full_size_c2_strong_split_bit_identical(built):
    """C2 split 8 ways (the strong-scaled multi-GPU split) with four lanes per pixel:
    the assembled frame equals the one-GPU one-lane frame bit for bit."""
    s, d, o = built["box"]
    W, H, spp, depth = 1920, 1080, 1024, 8
    pt = T.PathTracer("", W, H, 0)
    full = np.zeros((H, W, 3), np.float32)
    st = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=full)
    acc = np.zeros((H, W, 3), np.float32)
    rays = 0
    for r in range(8):
        st_r = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=acc, band=(16, 8, r),
                          lanes_per_pixel=4)
        rays += st_r["traversals"]
    assert _same(acc, full)
    assert rays == st["traversals"]


def test_auto_lanes_bit_identical_on_small_and_large_launches(built):
    """lanes_per_pixel 0 picks four lanes per pixel for launches with no more pixels
    than the chip's resident lanes (327,680) and one lane above: either way the
    one-lane frame, bit for bit, with the same rays."""
    s, d, o = built["box"]
    for W, H, spp in ((200, 120, 16), (1920, 1080, 2)):
        rad0, fb0, st0 = _render(s, d, W, H, spp, 8, None, 0)
        rad1, fb1, st1 = _render(s, d, W, H, spp, 8, None, 1)
        assert _same(rad0, rad1)
        assert np.array_equal(fb0, fb1)
        for k in STATS:
            assert st0[k] == st1[k], k
    acc = np.zeros((1080, 1920, 3), np.float32)   # the strong-scaled split at N = 8: four lanes (auto)
    for b in range(8):
        part, _, _ = _render(s, d, 1920, 1080, 2, 8, None, 0, band=(16, 8, b))
        rows = [y for y in range(1080) if (y // 16) % 8 == b]
        acc[rows] = part[rows]
    assert _same(acc, rad1)
