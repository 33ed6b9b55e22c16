"""GPU parity of the wavefront / ray-queue variant (TPT_FLAG_WAVEFRONT, wavefront.hip;
DESIGN.md section 5 "N1").

The variant cuts the reference's per-pixel loops (trace, path_tracer.cu:296-435)
at every traversal: a logic kernel runs the path logic of every queued ray and
compacts the next rays into a queue, a persistent trace kernel walks them.  Every
pixel's samples still run in order on its own XORWOW stream, so the frame must be
the megakernel's (k_trace) bit for bit, and the oracle's: every case below
compares all three, plus the ray counts.
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from oracle import oracle as O
from tests.conftest import scene_path
from tests.test_gpu_parity import CASES, assert_parity, image_metrics

pytestmark = pytest.mark.gpu

WF = T._lib.FLAG_WAVEFRONT
SCENES = ["box", "box1", "box2", "ball", "tir", "light", "square", "c5"]


@pytest.fixture(scope="module")
def built():
    out = {}
    for name in SCENES:
        s = T.Scene(scene_path(name))
        out[name] = (s, s.copySceneToDevice(0).build(), O.load_scene(scene_path(name)))
    yield out
    for _, d, _ in out.values():
        d.close()


def _render(s, d, W, H, spp, depth, env, flags=0, seed=42, **kw):
    pt = T.PathTracer("", W, H, 0)
    if env is not None:
        pt.envLight = T.EnvLight(env, 0)
    rad = np.zeros((H, W, 3), np.float32)
    fb = np.zeros((H, W, 4), np.uint8)
    st = pt.doTrace(d, s.m_camera, fb, spp, seed=seed, max_depth=depth, radiance=rad, flags=flags, **kw)
    return rad, fb, st


def _same(a, b):
    return np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.parametrize("order", ["ordered", "reference"])
@pytest.mark.parametrize("name,W,H,spp,depth,env", CASES)
def test_wavefront_matches_megakernel_and_oracle(built, name, W, H, spp, depth, env, order):
    s, d, o = built[name]
    sky = T.procedural_sky(64, 32) if env else None
    base = T._lib.FLAG_REF_ORDER if order == "reference" else 0
    mrad, mfb, mst = _render(s, d, W, H, spp, depth, sky, base)
    wrad, wfb, wst = _render(s, d, W, H, spp, depth, sky, base | WF)
    assert _same(wrad, mrad)
    assert np.array_equal(wfb, mfb)
    for k in ("traversals", "local_rays", "shade_hits", "pixels", "samples"):
        assert wst[k] == mst[k], k
    orad, obgra, oc = O.render(o, W, H, spp, depth, 42, env=sky[::-1].copy() if env else None, trig_mode=1)
    assert_parity(image_metrics(wrad, orad))
    assert np.array_equal(wfb[..., :3], obgra[..., :3])
    assert wst["traversals"] == oc["traversals"]


@pytest.mark.parametrize("slots", [256, 1024, 4096])
@pytest.mark.parametrize("name", ["box", "ball", "tir"])
def test_wavefront_slot_pool_bit_identical(built, name, slots):
    """Fewer slots than pixels: a slot runs one pixel's samples, stores it and claims
    the next pixel; the frame is the same."""
    s, d, o = built[name]
    sky = T.procedural_sky(64, 32) if name == "ball" else None
    W, H, spp, depth = 80, 44, 8, 16 if name == "tir" else 8
    mrad, _, mst = _render(s, d, W, H, spp, depth, sky)
    wrad, _, wst = _render(s, d, W, H, spp, depth, sky, WF, wf_slots=slots)
    assert _same(wrad, mrad)
    assert wst["traversals"] == mst["traversals"]


@pytest.mark.parametrize("refill", [1, 8, 40, 64])
def test_wavefront_refill_threshold_bit_identical(built, refill):
    s, d, o = built["box"]
    mrad, _, mst = _render(s, d, 96, 64, 8, 8, None)
    wrad, _, wst = _render(s, d, 96, 64, 8, 8, None, WF, wf_refill=refill)
    assert _same(wrad, mrad)
    assert wst["traversals"] == mst["traversals"]


@pytest.mark.parametrize("lanes", [1, 2])
def test_wavefront_env_importance_sampling(built, lanes):
    """A15 (opt-in env IS): the env shadow ray of every diffuse bounce is one more
    queued ray of the path; the megakernel in one-lane and pair mode agree."""
    s, d, o = built["ball"]
    sky = T.procedural_sky(256, 128)
    f = T._lib.FLAG_ENV_IS
    mrad, _, mst = _render(s, d, 64, 36, 16, 8, sky, f, lanes_per_pixel=lanes)
    wrad, _, wst = _render(s, d, 64, 36, 16, 8, sky, f | WF)
    assert _same(wrad, mrad)
    assert wst["traversals"] == mst["traversals"]


def test_wavefront_bands_frames_and_progressive(built):
    s, d, o = built["box"]
    W, H, spp = 64, 48, 8
    full, _, _ = _render(s, d, W, H, spp, 8, None, WF)
    # interleaved bands (multi-GPU sharding) assemble the same frame
    acc = np.zeros_like(full)
    for b in range(3):
        part, _, _ = _render(s, d, W, H, spp, 8, None, WF, band=(8, 3, b))
        rows = [y for y in range(H) if (y // 8) % 3 == b]
        acc[rows] = part[rows]
    assert _same(acc, full)
    # a batch of frames: frame f == a lone render with seed f
    pt = T.PathTracer("", W, H, 0)
    rads = [np.zeros((H, W, 3), np.float32) for _ in range(2)]
    pt.doTraceFrames(d, s.m_camera, [42, 43], None, spp, max_depth=8, radiances=rads, flags=WF)
    one43, _, _ = _render(s, d, W, H, spp, 8, None, 0, seed=43)
    assert _same(rads[0], full)
    assert _same(rads[1], one43)
    # progressive: 4 + 4 spp == 8 spp
    pt = T.PathTracer("", W, H, 0)
    r1 = np.zeros((H, W, 3), np.float32)
    pt.doTrace(d, s.m_camera, None, 4, seed=42, max_depth=8, radiance=r1, flags=WF)
    pt.doTrace(d, s.m_camera, None, 4, seed=42, max_depth=8, radiance=r1, flags=WF, accumulate=True)
    assert _same(r1, full)


@pytest.mark.parametrize("name,W,H,spp,depth,env", [
    ("box", 1920, 1080, 4, 8, None),
    ("ball", 1920, 1080, 2, 8, "sky"),
    ("tir", 1920, 1080, 4, 32, None),
    ("c5", 3840, 2160, 1, 8, None),
])
def test_wavefront_full_resolution_equals_megakernel(built, name, W, H, spp, depth, env):
    s, d, o = built[name]
    sky = T.procedural_sky(2048, 1024) if env else None
    mrad, mfb, mst = _render(s, d, W, H, spp, depth, sky)
    wrad, wfb, wst = _render(s, d, W, H, spp, depth, sky, WF)
    assert _same(wrad, mrad)
    assert np.array_equal(wfb, mfb)
    assert wst["traversals"] == mst["traversals"]
    assert wst["shade_hits"] == mst["shade_hits"]
