"""tpt_scene_build_async: the per-frame scene build whose host half (the SAH
traversal trees, wide_bvh.cpp) runs on a host thread while the render enqueues
its RNG initialisation (the reference rebuilds the BVH every frame before
setupRandSeed, path_tracer.cu:513,536-542).  The scene, and so every image,
must be the one tpt_scene_build makes, bit for bit, whatever the caller does
while the build is pending (render, trace single rays, rebuild, destroy).
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from tests.conftest import scene_path

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _render(d, scene, W=96, H=54, spp=4, seed=7):
    pt = T.PathTracer("", W, H, 0)
    rad = np.zeros((H, W, 3), np.float32)
    fb = np.zeros((H, W, 4), np.uint8)
    st = pt.doTrace(d, scene.m_camera, fb, spp, seed=seed, radiance=rad)
    return rad, fb, st


@pytest.mark.parametrize("name", ["box", "c5"])
def test_async_build_renders_like_sync(gpu_available, name):
    s = T.Scene(scene_path(name))
    a = s.copySceneToDevice(0)
    b = s.copySceneToDevice(0)
    try:
        ra, fa, sa = _render(a.build(), s)
        for threads in (-1, 1, 2):
            b.set_build_threads(threads)
            rb, fb, sb = _render(b.build(asynchronous=True), s)
            assert np.array_equal(_bits(ra), _bits(rb)), threads
            assert np.array_equal(fa, fb)
            for k in ("traversals", "wide_visits", "leaf_tests", "shade_hits"):
                assert sa[k] == sb[k], k
            assert sb["tree_wait_ms"] >= 0.0
        assert sa["tree_wait_ms"] == 0.0
    finally:
        a.close()
        b.close()


def test_async_build_superseded_and_destroyed_while_pending(gpu_available):
    s = T.Scene(scene_path("c5"))
    ref = s.copySceneToDevice(0).build()
    d = s.copySceneToDevice(0)
    try:
        ra, _, _ = _render(ref, s, seed=3)
        d.build(asynchronous=True)
        d.build(asynchronous=True)          # supersedes the pending one
        d.build()                           # and a synchronous build supersedes that
        rb, _, _ = _render(d, s, seed=3)
        assert np.array_equal(_bits(ra), _bits(rb))
        for _ in range(3):                  # a per-frame loop, as bench.py runs it
            d.build(asynchronous=True)
            rb, _, _ = _render(d, s, seed=3)
            assert np.array_equal(_bits(ra), _bits(rb))
    finally:
        ref.close()
        d.close()
    e = s.copySceneToDevice(0)
    e.build(asynchronous=True)
    e.close()                               # destroy joins the pending host build


def test_async_build_then_trace_rays(gpu_available):
    s = T.Scene(scene_path("c5"))
    a = s.copySceneToDevice(0).build()
    b = s.copySceneToDevice(0).build(asynchronous=True)
    try:
        rng = np.random.default_rng(5)
        o = rng.uniform(-1.0, 1.0, (512, 3)).astype(np.float32)
        dvec = rng.normal(size=(512, 3)).astype(np.float32)
        dvec /= np.linalg.norm(dvec, axis=1, keepdims=True)
        for mode in (0, 1):
            ha, ta, ua = a.trace_rays(o, dvec, mode=mode)
            hb, tb, ub = b.trace_rays(o, dvec, mode=mode)
            assert np.array_equal(ha, hb) and np.array_equal(_bits(ta), _bits(tb))
            assert np.array_equal(_bits(ua), _bits(ub))
    finally:
        a.close()
        b.close()
