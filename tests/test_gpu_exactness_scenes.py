"""GPU: exactness of the culled traversal on content its guards were not tuned on
(verdict r04 item 7; DESIGN.md section 4 "Culling").  The exactness scenes
(tinypathtracer_amd.synth.exactness_scene):
  x1s1, x1s2  box plus 12 randomly rotated, non-uniformly scaled, interpenetrating
              copies of its spheres, box2's cubes and light's icosphere (31,600
              triangles);
  x3          box, box1 and box2 with coplanar adjacent and coplanar overlapping
              walls (exact t ties decided by the leaf-position tie rule);
  x2          three boxes stacked exactly: duplicate Morton-key runs the
              reference's computeNodeRange (bvh.cu:150-217) turns into a cyclic
              parent chain -- the build must refuse it.
Against the oracle (bit for bit) and, at full size, the default traversal against
the reference's visit order (TPT_FLAG_REF_ORDER).  The TPT_VERIFY_CULL build's
ray-by-ray check of the same scenes is tools/gpu_verify.sh.
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from oracle import oracle as O
from tests.conftest import scene_path
from tests.test_gpu_parity import assert_parity, image_metrics

pytestmark = pytest.mark.gpu

SCENES = ["x1s1", "x1s2", "x3"]


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def built():
    out = {}
    for name in SCENES:
        s = T.Scene(scene_path(name))
        out[name] = (s, s.copySceneToDevice(0).build(), O.load_scene(scene_path(name)))
    yield out
    for _, d, _ in out.values():
        d.close()


@pytest.mark.parametrize("order", ["ordered", "reference"])
@pytest.mark.parametrize("name", SCENES)
def test_exactness_scene_matches_oracle(built, name, order):
    s, d, o = built[name]
    W, H, spp = 96, 54, 16
    pt = T.PathTracer("", W, H, 0)
    rad = np.zeros((H, W, 3), np.float32)
    fb = np.zeros((H, W, 4), np.uint8)
    flags = T._lib.FLAG_REF_ORDER if order == "reference" else 0
    st = pt.doTrace(d, s.m_camera, fb, spp, seed=42, max_depth=8, radiance=rad, flags=flags)
    orad, obgra, oc = O.render(o, W, H, spp, 8, 42, trig_mode=1)
    m = image_metrics(rad, orad)
    assert_parity(m)
    assert np.array_equal(fb[..., :3], obgra[..., :3])
    assert st["traversals"] == oc["traversals"]


@pytest.mark.parametrize("name", SCENES)
def test_exactness_scene_full_size_default_equals_reference_order(built, name):
    """1920x1080 x 64 spp: the culled ordered walk renders the reference order's frame."""
    s, d, o = built[name]
    W, H, spp = 1920, 1080, 64
    pt = T.PathTracer("", W, H, 0)
    a = np.zeros((H, W, 3), np.float32)
    b = np.zeros((H, W, 3), np.float32)
    sa = pt.doTrace(d, s.m_camera, None, spp, seed=7, max_depth=8, radiance=a)
    sb = pt.doTrace(d, s.m_camera, None, spp, seed=7, max_depth=8, radiance=b, flags=T._lib.FLAG_REF_ORDER)
    diff = int((_bits(a) != _bits(b)).any(-1).sum())
    assert diff == 0, diff
    assert sa["traversals"] == sb["traversals"]


def test_duplicate_key_topology_is_refused():
    s = T.Scene(scene_path("x2"))
    d = s.copySceneToDevice(0)
    with pytest.raises(T.TPTError, match="LBVH topology invalid"):
        d.build()
    d.close()
