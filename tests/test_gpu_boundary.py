"""The drop-in boundary with the reference's own device buffers.

The reference's doTrace holds only DeviceScene (mesh.cuh:80-96): thrust
device_vectors whose raw pointers are the `trace` kernel's arguments
(path_tracer.cu:297-299).  tpt_scene_create accepts those device pointers as
they are -- indices u32, Vec3 vertices/normals, Material, MtlInterval, Mat4
and the DeltaLight union (TPT_DESC_DELTALIGHT_LAYOUT) -- and must build and
render the same scene, bit for bit, as from the host arrays the glTF loader
produces.  INTEGRATION.md section 2 is the reference-side patch that does this.
"""
import copy

import numpy as np
import pytest

import tinypathtracer_amd as T
from tinypathtracer_amd import _lib
from tests.conftest import scene_path

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _render(d, scene, W=64, H=36, spp=8, env=None):
    pt = T.PathTracer("", W, H, 0)
    if env is not None:
        pt.envLight = T.EnvLight(env, 0)
    rad = np.zeros((H, W, 3), np.float32)
    fb = np.zeros((H, W, 4), np.uint8)
    st = pt.doTrace(d, scene.m_camera, fb, spp, seed=42, radiance=rad)
    return rad, fb, st


@pytest.mark.parametrize("name", ["box", "ball", "square", "tir"])
def test_scene_from_device_buffers_bit_identical(gpu_available, name):
    s = T.Scene(scene_path(name))
    host = s.copySceneToDevice(0).build()
    bufs = s.device_buffers(0)
    dev = T.DeviceScene(s, 0, buffers=bufs).build()
    try:
        for a, b in zip(host.read_world(), dev.read_world()):
            assert np.array_equal(_bits(a), _bits(b))
        (na, ka), (nb, kb) = host.read_bvh(), dev.read_bvh()
        assert np.array_equal(ka, kb) and na.tobytes() == nb.tobytes()
        sky = T.procedural_sky(64, 32) if name == "ball" else None
        ra, fa, sa = _render(host, s, env=sky)
        rb, fb, sb = _render(dev, s, env=sky)
        assert np.array_equal(_bits(ra), _bits(rb))
        assert np.array_equal(fa, fb)
        assert sa["traversals"] == sb["traversals"]
        if s.lights:
            assert ra.max() > 0.0
    finally:
        host.close()
        dev.close()


def test_deltalight_union_directional(gpu_available):
    """A directional light keeps its direction where the union's other members
    keep pos (delta_light.h:53-68 vs :35-51): the repacked union renders the
    same frame as the flat tpt_light, and the union's unowned bytes (NaN in
    Scene.device_buffers) are never read."""
    s = T.Scene(scene_path("box"))
    s2 = copy.copy(s)
    L = _lib.Light()
    L.type = 1
    L.color[:] = [1.0, 0.9, 0.8]
    L.intensity = 2.5
    L.direction[:] = [0.3, -0.9, -0.3]
    L.pos[:] = [0.0, 0.0, 0.0]
    spot = copy.copy(T.Scene(scene_path("square")).lights[0])
    s2.lights = [L, spot]
    host = s2.copySceneToDevice(0).build()
    dev = T.DeviceScene(s2, 0, buffers=s2.device_buffers(0)).build()
    try:
        ra, fa, sa = _render(host, s2)
        rb, fb, sb = _render(dev, s2)
        assert np.array_equal(_bits(ra), _bits(rb))
        assert np.array_equal(fa, fb)
        base, _, sc = _render(s.copySceneToDevice(0).build(), s)
        assert sa["traversals"] > sc["traversals"]          # the lights' shadow rays
        assert not np.array_equal(_bits(ra), _bits(base))    # and their light
    finally:
        host.close()
        dev.close()
