"""ctypes binding of libtpt.so (include/tpt.h).

The product path: every compute call goes through the HIP library.  If the
library is missing the import of this module raises -- there is no CPU
fallback (the CPU restatement in oracle/ is test infrastructure only).
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TPT_LIB", os.path.join(HERE, "libtpt.so"))

TPT_OK = 0
STATUS_NAMES = {0: "OK", 1: "INVALID_ARG", 2: "HIP_ERROR", 3: "OOM", 4: "IO", 5: "PARSE", 6: "NO_DEVICE"}
FLAG_NO_COUNTERS = 0x1
FLAG_REF_ORDER = 0x2
FLAG_ACCUMULATE = 0x4
FLAG_ENV_IS = 0x8
FLAG_APPROX_CULL = 0x10
FLAG_WAVEFRONT = 0x20
FLAG_FAST = 0x40
DESC_DELTALIGHT_LAYOUT = 0x1


class Material(C.Structure):
    _fields_ = [("base_color", C.c_float * 3), ("emission_factor", C.c_float), ("eta", C.c_float),
                ("metallic", C.c_float), ("subsurface", C.c_float), ("specular", C.c_float),
                ("roughness", C.c_float), ("specular_tint", C.c_float), ("anisotropic", C.c_float),
                ("sheen", C.c_float), ("sheen_tint", C.c_float), ("clearcoat", C.c_float),
                ("clearcoat_gloss", C.c_float)]


class Light(C.Structure):
    _fields_ = [("type", C.c_int32), ("color", C.c_float * 3), ("intensity", C.c_float),
                ("pos", C.c_float * 3), ("direction", C.c_float * 3), ("cos_outer", C.c_float),
                ("inv_cos_cone_diff", C.c_float)]


class Interval(C.Structure):
    _fields_ = [("begin", C.c_int32), ("mtl", C.c_int32)]


class SceneDesc(C.Structure):
    _fields_ = [("indices", C.POINTER(C.c_uint32)), ("n_faces", C.c_uint32),
                ("vertices", C.POINTER(C.c_float)), ("normals", C.POINTER(C.c_float)),
                ("n_vertices", C.c_uint32), ("lut", C.POINTER(Interval)), ("n_objects", C.c_uint32),
                ("vert_trans", C.POINTER(C.c_float)), ("normal_trans", C.POINTER(C.c_float)),
                ("materials", C.POINTER(Material)), ("n_materials", C.c_uint32),
                ("lights", C.POINTER(Light)), ("n_lights", C.c_uint32), ("flags", C.c_uint32)]


class Camera(C.Structure):
    _fields_ = [("c2w", C.c_float * 16), ("vfov", C.c_float), ("aspect", C.c_float), ("znear", C.c_float)]


class Params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32), ("max_depth", C.c_int32),
                ("seed", C.c_uint64), ("band_rows", C.c_int32), ("band_count", C.c_int32),
                ("band_index", C.c_int32), ("spp_per_launch", C.c_int32), ("flags", C.c_int32),
                ("refill", C.c_int32), ("pipe_sets", C.c_int32), ("pipe_chunks", C.c_int32),
                ("lanes_per_pixel", C.c_int32), ("leaf_batch", C.c_int32), ("wf_slots", C.c_int32),
                ("wf_refill", C.c_int32), ("band_list_len", C.c_int32), ("band_list", C.POINTER(C.c_int32)),
                ("band_cost", C.POINTER(C.c_float))]


class Stats(C.Structure):
    _fields_ = [("traversals", C.c_uint64), ("internal_visits", C.c_uint64), ("leaf_tests", C.c_uint64),
                ("shade_hits", C.c_uint64), ("pixels", C.c_uint64), ("samples", C.c_uint64),
                ("rng_init_ms", C.c_double), ("trace_ms", C.c_double), ("resolve_ms", C.c_double),
                ("total_ms", C.c_double), ("trace_launches", C.c_int32), ("pad", C.c_int32),
                ("wide_visits", C.c_uint64), ("accumulated_spp", C.c_uint64), ("trace_kernel_ms", C.c_double),
                ("local_rays", C.c_uint64), ("tree_wait_ms", C.c_double), ("resident_lanes", C.c_uint64),
                ("lanes_per_pixel", C.c_int32), ("drained", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "pad"}


# (name, restype, argtypes) -- every symbol include/tpt.h declares
SIGNATURES = [
    ("tpt_version", C.c_char_p, []),
    ("tpt_last_error", C.c_char_p, []),
    ("tpt_device_count", C.c_int, []),
    ("tpt_scene_create", C.c_int, [C.POINTER(SceneDesc), C.c_int, C.POINTER(C.c_void_p)]),
    ("tpt_scene_build", C.c_int, [C.c_void_p]),
    ("tpt_scene_build_async", C.c_int, [C.c_void_p]),
    ("tpt_scene_set_build_threads", C.c_int, [C.c_void_p, C.c_int32]),
    ("tpt_scene_destroy", None, [C.c_void_p]),
    ("tpt_env_create", C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.c_int, C.POINTER(C.c_void_p)]),
    ("tpt_env_destroy", None, [C.c_void_p]),
    ("tpt_env_load", C.c_int, [C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    ("tpt_image_load", C.c_int, [C.c_char_p, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_int32),
                                 C.POINTER(C.c_int32)]),
    ("tpt_image_free", None, [C.c_void_p]),
    ("tpt_render", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_void_p,
                             C.c_void_p, C.POINTER(Stats)]),
    ("tpt_render_frames", C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(Camera), C.POINTER(Params), C.c_int32,
                                    C.POINTER(C.c_uint64), C.POINTER(C.c_void_p), C.POINTER(C.c_void_p),
                                    C.POINTER(Stats)]),
    ("tpt_scene_read_bvh", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("tpt_scene_read_world", C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    ("tpt_debug_rng_init", C.c_int, [C.c_int, C.c_uint64, C.c_uint64, C.c_uint32, C.c_void_p]),
    ("tpt_debug_trace_rays", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                       C.c_void_p, C.c_void_p, C.c_void_p]),
    ("tpt_debug_hot_kat", C.c_int, [C.c_int, C.c_int32, C.c_uint32, C.c_void_p, C.c_void_p]),
    ("tpt_debug_step_latency", C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32,
                                         C.c_void_p]),
    ("tpt_wide_tree_build", C.c_int32, [C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32,
                                        C.POINTER(C.c_int32), C.c_int32]),
    ("tpt_gltf_load", C.c_int, [C.c_char_p, C.POINTER(C.c_void_p)]),
    ("tpt_gltf_desc", C.c_int, [C.c_void_p, C.POINTER(SceneDesc), C.POINTER(Camera)]),
    ("tpt_gltf_missing_material", C.c_int, [C.c_void_p]),
    ("tpt_gltf_free", None, [C.c_void_p]),
]


class TPTError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"tpt error {STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


_lib = None


def build_identity() -> dict:
    """The library this process runs: the SHA-256 (first 16 hex digits) of
    libtpt.so's bytes -- its code objects included -- and the git HEAD the
    Makefile recorded when it linked it (libtpt.build; "-dirty" when the tree
    had uncommitted changes).  bench.py prints it; tools/pmc_summary.py copies
    it into every PMC summary, so a bench line can tell whether its counters
    come from the same build."""
    import hashlib
    h = hashlib.sha256()
    with open(LIB_PATH, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    ident = {"lib_sha256": h.hexdigest()[:16], "git_head": None}
    try:
        with open(os.path.splitext(LIB_PATH)[0] + ".build") as f:
            ident["git_head"] = f.read().strip() or None
    except OSError:
        pass
    return ident


def lib():
    """Load libtpt.so (fails loudly when the HIP build is missing)."""
    global _lib
    if _lib is None:
        try:   # one HIP runtime per process: let torch's copy win the soname if present
            import torch  # noqa: F401
        except Exception:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"libtpt.so not found at {LIB_PATH}: build it with "
                              f"`make -C {HERE}` or __graft_entry__.build()")
        L = C.CDLL(LIB_PATH)
        # TPT_LIB (tools/gpu_abn.sh A/B of an older build) may name a library that
        # predates the newest debug entry points; the product library must export all
        older = bool(os.environ.get("TPT_LIB"))
        for name, res, args in SIGNATURES:
            if older and name.startswith("tpt_debug_") and not hasattr(L, name):
                continue
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(status):
    if status != TPT_OK:
        raise TPTError(status, lib().tpt_last_error().decode(errors="replace"))
