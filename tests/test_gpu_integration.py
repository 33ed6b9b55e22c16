"""The INTEGRATION.md reference-side patch across scene changes.

The patched PathTracer caches one tpt_scene handle (built from the reference's
DeviceScene device buffers) between doTrace frames.  render() may be called
again on the same PathTracer with another glTF (path_tracer.cu:556-579): it
builds a new DeviceScene, so the patch drops the handle in render() and
doTrace re-creates it for the DeviceScene it is handed (m_tptScene).  This
replays that caching logic over the same device-pointer path the patch uses
(Scene.device_buffers: DeviceScene's layouts) and checks every frame against
a fresh handle, bit for bit.
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from tests.conftest import scene_path

pytestmark = pytest.mark.gpu

W, H, SPP = 64, 36, 4


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


class PatchedPathTracer:
    """doTrace + render() with the cached handle."""

    def __init__(self, env=None):
        self.pt = T.PathTracer("", W, H, 0)
        if env is not None:
            self.pt.envLight = T.EnvLight(env, 0)
        self.m_tpt = None          # tpt_scene* m_tpt
        self.m_tptScene = None     # const DeviceScene* m_tptScene
        self.creates = 0

    def doTrace(self, d_scene, scene, seed):
        if self.m_tpt is not None and self.m_tptScene is not d_scene:   # another scene: stale handle
            self.m_tpt.close()
            self.m_tpt = None
        if self.m_tpt is None:
            self.m_tptScene = d_scene
            self.m_tpt = T.DeviceScene(scene, 0, buffers=d_scene)         # tpt_scene_create(device pointers)
            self.creates += 1
        self.m_tpt.build(asynchronous=True)                              # tpt_scene_build_async, every frame
        rad = np.zeros((H, W, 3), np.float32)
        fb = np.zeros((H, W, 4), np.uint8)
        self.pt.doTrace(self.m_tpt, scene.m_camera, fb, SPP, seed=seed, radiance=rad)
        return rad, fb

    def render(self, name, frames=2):
        scene = T.Scene(scene_path(name))
        d_scene = scene.device_buffers(0)       # DeviceScene d_scene = scene.copySceneToDevice()
        if self.m_tpt is not None:              # the patch's added line: a new scene drops the handle
            self.m_tpt.close()
            self.m_tpt = None
        return [self.doTrace(d_scene, scene, 42 + f) for f in range(frames)]

    def close(self):
        if self.m_tpt is not None:
            self.m_tpt.close()


def _fresh(name, seed, env=None):
    scene = T.Scene(scene_path(name))
    d = scene.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        if env is not None:
            pt.envLight = T.EnvLight(env, 0)
        rad = np.zeros((H, W, 3), np.float32)
        fb = np.zeros((H, W, 4), np.uint8)
        pt.doTrace(d, scene.m_camera, fb, SPP, seed=seed, radiance=rad)
        return rad, fb
    finally:
        d.close()


def test_scene_change_through_one_pathtracer(gpu_available):
    sky = T.procedural_sky(64, 32)
    p = PatchedPathTracer(env=sky)
    try:
        seq = ["box", "ball", "box"]
        for name in seq:
            frames = p.render(name)
            for f, (rad, fb) in enumerate(frames):
                ref_rad, ref_fb = _fresh(name, 42 + f, env=sky)
                assert np.array_equal(_bits(rad), _bits(ref_rad)), (name, f)
                assert np.array_equal(fb, ref_fb), (name, f)
        assert p.creates == len(seq)   # one handle per render(), kept across its frames
        # the scenes differ, so a stale handle would have shown
        a, _ = _fresh("box", 42, env=sky)
        b, _ = _fresh("ball", 42, env=sky)
        assert not np.array_equal(_bits(a), _bits(b))
    finally:
        p.close()
