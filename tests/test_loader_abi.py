"""CPU tests of the product's host side: the native glTF loader (libtpt.so,
tpt_gltf_*) against the oracle's restatement of mesh.cu, SURVEY Appendix C
scene facts, error behaviour, and the C-ABI surface (every symbol include/tpt.h
declares is exported; struct layouts match the header)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import tinypathtracer_amd as T
from tinypathtracer_amd import _lib
from oracle import scene as S
from tests.conftest import ROOT, scene_path

ALL = ["ball", "box", "box1", "box2", "light", "square", "tir"]


def _u(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("name", ALL)
def test_native_loader_matches_oracle_bit_exact(name):
    a = T.Scene(scene_path(name))
    b = S.load_gltf(scene_path(name))
    assert np.array_equal(a.indices, b.indices)
    assert np.array_equal(_u(a.vertices), _u(b.vertices))
    assert np.array_equal(_u(a.normals), _u(b.normals))
    assert np.array_equal(a.lut, b.lut)
    assert np.array_equal(_u(a.vert_trans), _u(b.vert_trans))
    assert np.array_equal(_u(a.normal_trans), _u(b.normal_trans))
    assert np.array_equal(_u(a.materials), _u(b.materials))
    assert np.array_equal(_u(a.m_camera.c2w), _u(b.camera_c2w))
    assert np.float32(a.m_camera.vfov) == b.vfov and np.float32(a.m_camera.aspect) == b.aspect
    assert a.missing_material == b.missing_material
    assert len(a.lights) == len(b.lights)
    for la, lb in zip(a.lights, b.lights):
        assert la.type == lb["type"]
        assert np.float32(la.intensity) == lb["intensity"]
        assert list(_u(np.array(la.pos[:]))) == list(_u(np.array(lb["pos"])))
        assert list(_u(np.array(la.direction[:]))) == list(_u(np.array(lb["direction"])))
        assert np.float32(la.cos_outer) == lb["cos_outer"]
        assert np.float32(la.inv_cos_cone_diff) == lb["inv_cos_cone_diff"]


# SURVEY.md Appendix C (reference loader facts)
APPENDIX_C = {
    "box": dict(faces=1932, verts=1142, objects=8, lights=0, yfov=0.3996,
                mats=["blueWall", "glassBall", "glossyBall", "redWall", "squareLIght", "whitWall"]),
    "box1": dict(faces=10, verts=20, objects=5, lights=0, yfov=0.3996, mats=["blueWall", "redWall", "whitWall"]),
    "box2": dict(faces=36, verts=72, objects=8, lights=0, yfov=0.3996),
    "light": dict(faces=80, verts=240, objects=1, lights=0, yfov=0.3996, mats=["Material"]),
    "ball": dict(faces=1216, verts=660, objects=1, lights=1, yfov=1.0398, mats=[]),
    "tir": dict(faces=6, verts=12, objects=3, lights=0, yfov=1.0458,
                mats=["Material.001", "Material.002", "Material.003"]),
    "square": dict(faces=8, verts=16, objects=4, lights=1, yfov=1.0472, mats=[]),
}


@pytest.mark.parametrize("name", ALL)
def test_appendix_c_scene_facts(name):
    f = APPENDIX_C[name]
    s = T.Scene(scene_path(name))
    o = S.load_gltf(scene_path(name))
    assert s.n_faces == f["faces"]
    assert len(s.vertices) == f["verts"]
    assert len(s.lut) == f["objects"]
    assert len(s.lights) == f["lights"]
    assert round(float(s.m_camera.vfov), 4) == f["yfov"]
    assert abs(float(s.m_camera.aspect) - 1.7778) < 1e-4
    if "mats" in f:
        assert o.material_names == f["mats"]
    if name == "box":   # App. A.8: tinygltf default metallic = 1 -> glossyBall/whitWall semantics
        mats = dict(zip(o.material_names, o.materials))
        assert mats["glossyBall"][5] == 1.0            # metallic default
        assert mats["glassBall"][4] == 2.0             # eta from KHR_materials_ior
        assert mats["squareLIght"][3] == 6.0           # emissive strength
    if name in ("ball", "square"):                     # App. A.9: no material -> Material()
        assert s.missing_material


def test_light_units():
    s = T.Scene(scene_path("ball"))
    L = s.lights[0]
    assert L.type == 0 and np.float32(L.intensity) == np.float32(np.float32(1630.5423919764678) *
                                                                 np.float32(np.float32(1.0) / np.float32(683.0)))
    sq = T.Scene(scene_path("square")).lights[0]
    assert sq.type == 2 and sq.cos_outer > 0.9


def test_loader_errors(tmp_path):
    with pytest.raises(T.TPTError) as e:
        T.Scene(str(tmp_path / "missing.gltf"))
    assert e.value.status == 4                         # TPT_ERR_IO
    bad = tmp_path / "bad.gltf"
    bad.write_text("{ not json")
    with pytest.raises(T.TPTError) as e:
        T.Scene(str(bad))
    assert e.value.status == 5                         # TPT_ERR_PARSE
    with pytest.raises(RuntimeError):
        T.Scene(scene_path("box"), "obj")              # Scene(file, type) rejects non-gltf (mesh.cu:76)
    light_type = tmp_path / "light_type.gltf"
    src = open(scene_path("ball")).read().replace('"type":"point"', '"type":"area"')
    light_type.write_text(src)
    with pytest.raises(T.TPTError):
        T.Scene(str(light_type))                       # "Unsupported light type" (mesh.cu:303)


def _declared_symbols():
    src = open(os.path.join(ROOT, "include", "tpt.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tpt_[a-z_0-9]+)\s*\(", src)))


def test_abi_exports_every_declared_symbol():
    L = T.lib()
    declared = _declared_symbols()
    assert len(declared) >= 17
    for name in declared:
        assert hasattr(L, name), name
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(declared) == bound


def test_abi_struct_layouts(tmp_path):
    """ctypes mirrors vs the C compiler's layout of include/tpt.h."""
    prog = tmp_path / "layout.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "tpt.h"\n'
                    'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu\\n",'
                    'sizeof(tpt_material),sizeof(tpt_light),sizeof(tpt_interval),sizeof(tpt_scene_desc),'
                    'sizeof(tpt_camera),sizeof(tpt_params),sizeof(tpt_stats),offsetof(tpt_params,seed));return 0;}')
    exe = tmp_path / "layout"
    import subprocess
    subprocess.check_call(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)])
    sizes = [int(x) for x in subprocess.check_output([str(exe)]).split()]
    mine = [C.sizeof(_lib.Material), C.sizeof(_lib.Light), C.sizeof(_lib.Interval), C.sizeof(_lib.SceneDesc),
            C.sizeof(_lib.Camera), C.sizeof(_lib.Params), C.sizeof(_lib.Stats), _lib.Params.seed.offset]
    assert sizes == mine
    assert sizes[0] == 60 and sizes[1] == 52          # Material (material.h:86-120), DeltaLight 52 B
    assert T.NODE_DTYPE.itemsize == 36                # BVHNode (bvh.cuh:52-58)


def test_abi_without_device_fails_cleanly():
    if T.device_count() > 0:
        pytest.skip("a HIP device is visible")
    s = T.Scene(scene_path("tir"))
    with pytest.raises(T.TPTError) as e:
        s.copySceneToDevice(0)
    assert e.value.status == 6                         # TPT_ERR_NO_DEVICE
    h = C.c_void_p()
    assert T.lib().tpt_env_create(None, 0, 0, 0, C.byref(h)) == 1
    assert b"bad env" in T.lib().tpt_last_error()


def test_version_string():
    assert "gfx950" in T.version()
