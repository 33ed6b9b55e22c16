"""ctypes front end for liboracle.so -- TEST INFRASTRUCTURE ONLY.

The C oracle (tpt_oracle.c) restates the reference hot path; this module
loads it and feeds it scenes from oracle/scene.py.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from . import scene as oscene

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class Material(C.Structure):
    _fields_ = [("v", C.c_float * 15)]


class Light(C.Structure):
    _fields_ = [("type", C.c_int32), ("color", C.c_float * 3), ("intensity", C.c_float),
                ("pos", C.c_float * 3), ("direction", C.c_float * 3), ("cos_outer", C.c_float),
                ("inv_cos_cone_diff", C.c_float)]


class Interval(C.Structure):
    _fields_ = [("begin", C.c_int32), ("mtl", C.c_int32)]


class Scene(C.Structure):
    _fields_ = [("indices", C.POINTER(C.c_uint32)), ("n_faces", C.c_uint32),
                ("vertices", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("n_vertices", C.c_uint32),
                ("lut", C.POINTER(Interval)), ("n_objects", C.c_uint32),
                ("vert_trans", C.POINTER(C.c_float)), ("normal_trans", C.POINTER(C.c_float)),
                ("materials", C.POINTER(Material)), ("n_materials", C.c_uint32),
                ("lights", C.POINTER(Light)), ("n_lights", C.c_uint32)]


class Node(C.Structure):
    _fields_ = [("parent", C.c_uint32), ("a", C.c_int32), ("b", C.c_int32),
                ("bmin", C.c_float * 3), ("bmax", C.c_float * 3)]


class Env(C.Structure):
    _fields_ = [("rgba", C.POINTER(C.c_uint8)), ("w", C.c_int32), ("h", C.c_int32)]


class Camera(C.Structure):
    _fields_ = [("c2w", C.c_float * 16), ("vfov", C.c_float), ("aspect", C.c_float)]


class Params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32),
                ("max_depth", C.c_int32), ("seed", C.c_uint64), ("band_rows", C.c_int32),
                ("band_count", C.c_int32), ("band_index", C.c_int32), ("trig_mode", C.c_int32),
                ("threads", C.c_int32), ("env_is", C.c_int32)]


class Counters(C.Structure):
    _fields_ = [("traversals", C.c_uint64), ("internal_visits", C.c_uint64),
                ("leaf_tests", C.c_uint64), ("shade_hits", C.c_uint64), ("pixels", C.c_uint64),
                ("init_ms", C.c_double), ("trace_ms", C.c_double)]


_lib = None


def build():
    """Compile liboracle.so (gcc) if missing or stale."""
    src = [os.path.join(HERE, f) for f in ("tpt_oracle.c", "tpt_oracle.h")]
    if os.path.exists(LIB_PATH) and all(os.path.getmtime(LIB_PATH) >= os.path.getmtime(s) for s in src):
        return LIB_PATH
    subprocess.check_call(["make", "-C", HERE, "liboracle.so"], stdout=subprocess.DEVNULL)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_render.argtypes = [C.POINTER(Scene), C.POINTER(Env), C.POINTER(Camera), C.POINTER(Params),
                                 C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.POINTER(Counters)]
        L.orc_render.restype = C.c_int
        L.orc_build_bvh.argtypes = [C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_uint32),
                                    C.POINTER(Node), C.POINTER(C.c_int64)]
        L.orc_build_bvh.restype = C.c_int
        L.orc_transform.argtypes = [C.POINTER(Scene), C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.orc_xorwow_init.argtypes = [C.c_uint64, C.c_uint64, C.POINTER(C.c_uint32)]
        L.orc_env_is_samples.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_float), C.c_uint64, C.c_int,
                                         C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.orc_env_is_samples.restype = C.c_int
        L.orc_xorwow_next.argtypes = [C.POINTER(C.c_uint32)]
        L.orc_xorwow_next.restype = C.c_uint32
        L.orc_uniform.argtypes = [C.POINTER(C.c_uint32)]
        L.orc_uniform.restype = C.c_float
        L.orc_xorwow_jump_matrices.restype = C.POINTER(C.c_uint32)
        L.orc_float_to_21int.argtypes = [C.c_float]
        L.orc_float_to_21int.restype = C.c_int64
        L.orc_morton.argtypes = [C.c_float, C.c_float, C.c_float]
        L.orc_morton.restype = C.c_int64
        L.orc_set_x86_shift.argtypes = [C.c_int]
        L.orc_trace_ray.argtypes = [C.POINTER(Node), C.c_uint32, C.POINTER(C.c_float), C.POINTER(C.c_uint32),
                                    C.POINTER(C.c_float), C.POINTER(C.c_float), C.POINTER(C.c_float),
                                    C.POINTER(C.c_float)]
        L.orc_trace_ray.restype = C.c_int
        _lib = L
    return _lib


def use_library(path):
    """Load the oracle from another build of tpt_oracle.c (bench.py's CPU
    baseline: -O3 -march=native for the host), or back to liboracle.so (None)."""
    global _lib
    _lib = None
    if path:
        saved = globals()["LIB_PATH"]
        globals()["LIB_PATH"] = path
        try:
            lib()
        finally:
            globals()["LIB_PATH"] = saved


def _ptr(a, ct):
    return a.ctypes.data_as(C.POINTER(ct))


class PackedScene:
    """Keeps numpy buffers alive behind an orc_scene struct."""

    def __init__(self, s: oscene.OracleScene):
        self.src = s
        self.indices = np.ascontiguousarray(s.indices, dtype=np.uint32)
        self.vertices = np.ascontiguousarray(s.vertices, dtype=np.float32)
        self.normals = np.ascontiguousarray(s.normals, dtype=np.float32)
        self.lut = (Interval * max(len(s.lut), 1))(*[Interval(int(b), int(m)) for b, m in s.lut])
        self.vt = np.ascontiguousarray(s.vert_trans, dtype=np.float32)
        self.nt = np.ascontiguousarray(s.normal_trans, dtype=np.float32)
        nm = len(s.materials)
        self.mats = (Material * max(nm, 1))()
        for i in range(nm):
            self.mats[i].v[:] = [float(x) for x in s.materials[i]]
        nl = len(s.lights)
        self.lights = (Light * max(nl, 1))()
        for i, d in enumerate(s.lights):
            L = self.lights[i]
            L.type = d["type"]
            L.color[:] = [float(x) for x in d["color"]]
            L.intensity = float(d["intensity"])
            L.pos[:] = [float(x) for x in d["pos"]]
            L.direction[:] = [float(x) for x in d["direction"]]
            L.cos_outer = float(d["cos_outer"])
            L.inv_cos_cone_diff = float(d["inv_cos_cone_diff"])
        self.struct = Scene(_ptr(self.indices, C.c_uint32), len(self.indices) // 3,
                            _ptr(self.vertices, C.c_float), _ptr(self.normals, C.c_float),
                            len(self.vertices),
                            C.cast(self.lut, C.POINTER(Interval)), len(s.lut),
                            _ptr(self.vt, C.c_float), _ptr(self.nt, C.c_float),
                            C.cast(self.mats, C.POINTER(Material)), nm,
                            C.cast(self.lights, C.POINTER(Light)), nl)


def load_scene(path):
    return PackedScene(oscene.load_gltf(path))


def transform(ps: PackedScene):
    nv = len(ps.vertices)
    wv = np.zeros((nv, 3), np.float32)
    wn = np.zeros((nv, 3), np.float32)
    lib().orc_transform(C.byref(ps.struct), _ptr(wv, C.c_float), _ptr(wn, C.c_float))
    return wv, wn


def build_bvh(ps: PackedScene):
    """Returns (nodes structured array, sorted keys, world verts, world normals)."""
    wv, wn = transform(ps)
    nf = len(ps.indices) // 3
    nodes = (Node * (2 * nf - 1))()
    keys = np.zeros(nf, np.int64)
    rc = lib().orc_build_bvh(nf, _ptr(wv, C.c_float), _ptr(ps.indices, C.c_uint32), nodes,
                             _ptr(keys, C.c_int64))
    if rc == -3:
        raise ValueError("LBVH topology invalid: a parent chain misses the root (duplicate Morton keys)")
    assert rc == 0
    arr = np.frombuffer(nodes, dtype=np.dtype([("parent", "<u4"), ("a", "<i4"), ("b", "<i4"),
                                               ("bmin", "<f4", 3), ("bmax", "<f4", 3)])).copy()
    return arr, keys, wv, wn


def topology_hash(nodes, n_faces):
    """FNV-1a 64 over (left, right) of internal nodes, then leaf fids."""
    h = 0xcbf29ce484222325
    P = 0x100000001b3
    M = (1 << 64) - 1

    def feed(v):
        nonlocal h
        for byte in int(v & 0xffffffff).to_bytes(4, "little"):
            h ^= byte
            h = (h * P) & M

    for i in range(n_faces - 1):
        feed(int(nodes["a"][i]))
        feed(int(nodes["b"][i]))
    for j in range(n_faces - 1, 2 * n_faces - 1):
        feed(int(nodes["a"][j]))
    return h


def render(ps: PackedScene, width, height, spp, max_depth=8, seed=42, env=None, trig_mode=1,
           band_rows=0, band_count=1, band_index=0, threads=0, cam=None, env_is=False):
    """Run the oracle frame.  env: (rgba uint8 [h,w,4] row0=bottom) or None.
    Returns (radiance [H,W,3] row0=bottom, bgra [H,W,4] row0=top, counters dict)."""
    s = ps.src
    camera = Camera()
    camera.c2w[:] = [float(x) for x in (cam["c2w"] if cam else s.camera_c2w)]
    camera.vfov = float(cam["vfov"] if cam else s.vfov)
    camera.aspect = float(cam["aspect"] if cam else s.aspect)
    p = Params(width, height, spp, max_depth, seed, band_rows, band_count, band_index, trig_mode, threads,
               1 if env_is else 0)
    rad = np.zeros((height, width, 3), np.float32)
    bgra = np.zeros((height, width, 4), np.uint8)
    cnt = Counters()
    envp = None
    if env is not None:
        env = np.ascontiguousarray(env, dtype=np.uint8)
        envs = Env(_ptr(env, C.c_uint8), env.shape[1], env.shape[0])
        envp = C.byref(envs)
    rc = lib().orc_render(C.byref(ps.struct), envp, C.byref(camera), C.byref(p),
                          _ptr(rad, C.c_float), _ptr(bgra, C.c_uint8), C.byref(cnt))
    if rc != 0:
        raise RuntimeError(f"orc_render failed: {rc}")
    counters = {k: getattr(cnt, k) for k, _ in Counters._fields_}
    return rad, bgra, counters


def xorwow_stream(seed, subsequence, n):
    st = (C.c_uint32 * 6)()
    lib().orc_xorwow_init(seed, subsequence, st)
    return [lib().orc_xorwow_next(st) for _ in range(n)]


def uniform_stream(seed, subsequence, n):
    st = (C.c_uint32 * 6)()
    lib().orc_xorwow_init(seed, subsequence, st)
    return np.array([lib().orc_uniform(st) for _ in range(n)], np.float32)


def jump_matrices():
    p = lib().orc_xorwow_jump_matrices()
    return np.ctypeslib.as_array(p, shape=(32 * 160 * 5,)).reshape(32, 160, 5).copy()


def env_is_samples(rgba_bottom_up, nf, n, seed=7):
    """n env importance samples (the build's A15 re-derivation) for normal nf:
    (dirs [n,3], contribution factors Le*cos/(pi*pdf) [n,3])."""
    rgba = np.ascontiguousarray(rgba_bottom_up, np.uint8)
    h, w = rgba.shape[:2]
    d = np.zeros((n, 3), np.float32)
    k = np.zeros((n, 3), np.float32)
    nfa = (C.c_float * 3)(*[float(x) for x in nf])
    rc = lib().orc_env_is_samples(rgba.ctypes.data, w, h, nfa, seed, n, _ptr(d, C.c_float), _ptr(k, C.c_float))
    assert rc == 0
    return d, k
