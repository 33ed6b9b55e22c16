"""tinypathtracer_amd -- MI355X-native TinyPathTracer hot path, Python host mirror.

Mirrors the reference host API (include/path_tracer.h:16-35,
include/mesh.cuh:98-115, include/bvh.cuh:60-68, include/camera.h) over the
C-ABI in include/tpt.h (libtpt.so, HIP for gfx950):

    pt = PathTracer(env_file)            # PathTracer(const std::string&)
    frame = pt.render("input/box.gltf")  # render(meshFile), headless

Scene/Mesh loading, BVH construction and the trace megakernel all run in the
native library; this module only marshals arrays.
"""
from __future__ import annotations

import ctypes as C
import os
import time
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import TPTError, build_identity, check, lib

__all__ = ["Camera", "Scene", "DeviceScene", "BVH", "EnvLight", "PathTracer", "Frame", "TPTError",
           "procedural_sky", "version", "device_count", "build_identity", "NODE_DTYPE"]

# BVHNode (include/bvh.cuh:52-58): parent, info{left,right | fid,placeHolder}, box
NODE_DTYPE = np.dtype([("parent", "<u4"), ("a", "<i4"), ("b", "<i4"), ("bmin", "<f4", 3), ("bmax", "<f4", 3)])


def version() -> str:
    return lib().tpt_version().decode()


def device_count() -> int:
    return int(lib().tpt_device_count())


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


@dataclass
class Camera:
    """include/camera.h:9-65 (getters :56-58); c2w = m_transform->localToWorld()."""
    c2w: np.ndarray
    vfov: float
    aspect: float
    znear: float = 0.1

    def getVFov(self):
        return self.vfov

    def getAspRatio(self):
        return self.aspect

    def getNearPlane(self):
        return self.znear

    def to_c(self) -> _lib.Camera:
        c = _lib.Camera()
        c.c2w[:] = [float(v) for v in np.asarray(self.c2w, np.float32).reshape(16)]
        c.vfov, c.aspect, c.znear = float(self.vfov), float(self.aspect), float(self.znear)
        return c


class Scene:
    """Scene(filename, type) (mesh.cu:68-79): host-side glTF scene, loaded by the
    native loader (mesh.cu:80-307 semantics).  Arrays are the packed content of
    copySceneToDevice (mesh.cu:309-397)."""

    def __init__(self, filename: str, type: str = "gltf"):
        if type != "gltf":
            raise RuntimeError("Unsupported file format. Only support .gltf file.")
        h = C.c_void_p()
        check(lib().tpt_gltf_load(os.fsencode(filename), C.byref(h)))
        try:
            d = _lib.SceneDesc()
            cam = _lib.Camera()
            check(lib().tpt_gltf_desc(h, C.byref(d), C.byref(cam)))
            nf, nv = d.n_faces, d.n_vertices
            self.indices = np.ctypeslib.as_array(d.indices, (3 * nf,)).copy()
            self.vertices = np.ctypeslib.as_array(d.vertices, (nv, 3)).copy()
            self.normals = np.ctypeslib.as_array(d.normals, (nv, 3)).copy()
            self.lut = np.array([(d.lut[i].begin, d.lut[i].mtl) for i in range(d.n_objects)], np.int32)
            self.vert_trans = np.ctypeslib.as_array(d.vert_trans, (d.n_objects, 16)).copy()
            self.normal_trans = np.ctypeslib.as_array(d.normal_trans, (d.n_objects, 16)).copy()
            self.materials = np.array([[*d.materials[i].base_color] + [getattr(d.materials[i], f)
                                        for f, _ in _lib.Material._fields_[1:]] for i in range(d.n_materials)],
                                      np.float32).reshape(-1, 15)
            self.lights = [_lib.Light.from_buffer_copy(d.lights[i]) for i in range(d.n_lights)]
            self.missing_material = bool(lib().tpt_gltf_missing_material(h))
            self.m_camera = Camera(np.array(cam.c2w[:], np.float32), cam.vfov, cam.aspect, cam.znear)
        finally:
            lib().tpt_gltf_free(h)
        self.filename = filename

    @property
    def n_faces(self):
        return len(self.indices) // 3

    def desc(self):
        """tpt_scene_desc view (keeps buffers alive on self)."""
        self._mats = (_lib.Material * max(len(self.materials), 1))()
        for i, row in enumerate(self.materials):
            m = self._mats[i]
            m.base_color[:] = [float(v) for v in row[:3]]
            for k, (f, _) in enumerate(_lib.Material._fields_[1:]):
                setattr(m, f, float(row[3 + k]))
        self._lights = (_lib.Light * max(len(self.lights), 1))(*self.lights)
        self._lut = (_lib.Interval * len(self.lut))(*[_lib.Interval(int(b), int(m)) for b, m in self.lut])
        self._arr = [np.ascontiguousarray(a) for a in (self.indices, self.vertices, self.normals,
                                                        self.vert_trans, self.normal_trans)]
        ind, ver, nor, vt, nt = self._arr
        return _lib.SceneDesc(
            ind.ctypes.data_as(C.POINTER(C.c_uint32)), self.n_faces,
            ver.ctypes.data_as(C.POINTER(C.c_float)), nor.ctypes.data_as(C.POINTER(C.c_float)), len(ver),
            C.cast(self._lut, C.POINTER(_lib.Interval)), len(self.lut),
            vt.ctypes.data_as(C.POINTER(C.c_float)), nt.ctypes.data_as(C.POINTER(C.c_float)),
            C.cast(self._mats, C.POINTER(_lib.Material)), len(self.materials),
            C.cast(self._lights, C.POINTER(_lib.Light)), len(self.lights))

    def copySceneToDevice(self, device: int = 0) -> "DeviceScene":
        return DeviceScene(self, device)

    def device_buffers(self, device: int = 0) -> dict:
        """The reference's DeviceScene (mesh.cuh:80-96) as torch tensors in HBM of
        `device`, element types and layouts as the reference's thrust
        device_vectors hold them: indices u32, Vec3 vertices/normals, Material
        (15 floats), MtlInterval, column-major Mat4, and DeltaLight
        (delta_light.h:96-130, 52 B: the type, then the light union -- a
        directional light's direction where the others keep pos; bytes a light
        type does not own are NaN here, so a reader of them would show).  These
        are the `trace` kernel's own arguments (path_tracer.cu:297-299);
        DeviceScene(scene, device, buffers=...) hands them to tpt_scene_create
        as device pointers."""
        import torch
        dev = torch.device("cuda", device)
        lights = np.full((max(len(self.lights), 1), 13), np.nan, np.float32)
        for i, L in enumerate(self.lights):
            row = lights[i]
            row[0:1].view(np.int32)[0] = L.type
            row[1:4] = L.color[:]
            row[4] = L.intensity
            if L.type == 1:    # DirectionalLight{color, intensity, direction}
                row[5:8] = L.direction[:]
            else:              # PointLight{color, intensity, pos}; SpotLight{..., pos, direction, cos, invDiff}
                row[5:8] = L.pos[:]
                if L.type == 2:
                    row[8:11] = L.direction[:]
                    row[11] = L.cos_outer
                    row[12] = L.inv_cos_cone_diff
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev) if len(a) else \
            torch.empty(0, dtype=dt, device=dev)
        bufs = {
            "indices": t(self.indices.astype(np.uint32).view(np.int32), torch.int32),
            "vertices": t(self.vertices.astype(np.float32), torch.float32),
            "normals": t(self.normals.astype(np.float32), torch.float32),
            "materials": t(self.materials.astype(np.float32), torch.float32),
            "materialsLUT": t(self.lut.astype(np.int32), torch.int32),
            "vertTrans": t(self.vert_trans.astype(np.float32), torch.float32),
            "normalTrans": t(self.normal_trans.astype(np.float32), torch.float32),
            "lights": t(lights[:len(self.lights)], torch.float32),
        }
        torch.cuda.synchronize(dev)
        return bufs


class DeviceScene:
    """DeviceScene (mesh.cuh:80-96): scene buffers resident in HBM of `device`."""

    def __init__(self, scene: Scene, device: int = 0, buffers: dict | None = None):
        """buffers: Scene.device_buffers() -- device arrays in the reference's
        layouts, passed to tpt_scene_create as device pointers (the reference's
        doTrace hands over its DeviceScene this way)."""
        self.scene = scene
        self.device = device
        self.handle = C.c_void_p()
        if buffers is None:
            d = scene.desc()
        else:
            b = buffers
            dp = lambda k, ty: C.cast(C.c_void_p(b[k].data_ptr() if b[k].numel() else 0), C.POINTER(ty))
            d = _lib.SceneDesc(
                dp("indices", C.c_uint32), b["indices"].numel() // 3,
                dp("vertices", C.c_float), dp("normals", C.c_float), b["vertices"].numel() // 3,
                dp("materialsLUT", _lib.Interval), b["materialsLUT"].numel() // 2,
                dp("vertTrans", C.c_float), dp("normalTrans", C.c_float),
                dp("materials", _lib.Material), b["materials"].numel() // 15,
                dp("lights", _lib.Light), b["lights"].numel() // 13, _lib.DESC_DELTALIGHT_LAYOUT)
        check(lib().tpt_scene_create(C.byref(d), device, C.byref(self.handle)))
        self.built = False

    def set_build_threads(self, threads: int):
        """Host threads of the traversal-tree build (tpt_scene_set_build_threads):
        < 0 the usable cores, 0/1 serial; the same tree either way."""
        check(lib().tpt_scene_set_build_threads(self.handle, int(threads)))
        return self

    def build(self, asynchronous: bool = False):
        """World transform + LBVH (path_tracer.cu:536-542) on the device, then
        the host SAH traversal trees.  asynchronous=True: the host trees finish
        on a background thread (tpt_scene_build_async) while the next render
        enqueues its RNG initialisation; that render waits for them."""
        check(lib().tpt_scene_build_async(self.handle) if asynchronous else lib().tpt_scene_build(self.handle))
        self.built = True
        return self

    def read_bvh(self):
        nf = self.scene.n_faces
        nodes = np.zeros(2 * nf - 1, NODE_DTYPE)
        keys = np.zeros(nf, np.int64)
        check(lib().tpt_scene_read_bvh(self.handle, _ptr(nodes), _ptr(keys)))
        return nodes, keys

    def read_world(self):
        nv = len(self.scene.vertices)
        wv = np.zeros((nv, 3), np.float32)
        wn = np.zeros((nv, 3), np.float32)
        check(lib().tpt_scene_read_world(self.handle, _ptr(wv), _ptr(wn)))
        return wv, wn

    def trace_rays(self, origins, dirs, mode=0, origin_fid=None):
        """mode 0: the reference's visit order; 1: the render's ordered culled
        traversal; 2: any hit; 3: two-pass probe (see tpt_debug_trace_rays).
        origin_fid: per ray the face it leaves (-1 none), as the render knows it
        for secondary rays (the grazing test)."""
        o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        n = len(o)
        hit = np.zeros(n, np.int32)
        t = np.zeros(n, np.float32)
        uv = np.zeros((n, 2), np.float32)
        of = None if origin_fid is None else np.ascontiguousarray(origin_fid, np.int32).reshape(n)
        check(lib().tpt_debug_trace_rays(self.handle, n, _ptr(o), _ptr(d), _ptr(of), mode, _ptr(hit), _ptr(t),
                                         _ptr(uv)))
        return hit, t, uv

    def step_latency(self, origins, dirs, mode=0, flags=0):
        """ONE 64-lane wave walks these <= 64 closest-hit rays (tpt_debug_step_latency):
        mode 0 nodes from global memory, 1 the whole 4-wide tree in LDS, 2 four lanes
        per ray (<= 16 rays; steps = node visits, leaf children tested in-node).  Returns
        (steps per lane, wave loop iterations, wave shader cycles, hit fids)."""
        o = np.ascontiguousarray(origins, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(dirs, np.float32).reshape(-1, 3)
        out = np.zeros((64, 4), np.uint64)
        check(lib().tpt_debug_step_latency(self.handle, len(o), _ptr(o), _ptr(d), mode, flags, _ptr(out)))
        n = len(o)
        return out[:n, 0].astype(np.int64), int(out[0, 1]), int(out[0, 2]), out[:n, 3].astype(np.int64)

    def close(self):
        if self.handle:
            lib().tpt_scene_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def hot_kat(op, cases, device=0):
    """The trace kernel's own device functions on `cases` (tpt_debug_hot_kat):
    op 0 box (n,12) -> (n,2); 1 triangle (n,15) -> (n,4); 2 light (n,16) -> (n,6);
    3 toUChar (n,3) -> (n,3).  Tests pin them to the reference's headers."""
    nin, nout = {0: (12, 2), 1: (15, 4), 2: (16, 6), 3: (3, 3)}[op]
    a = np.ascontiguousarray(cases, np.float32).reshape(-1, nin)
    out = np.zeros((len(a), nout), np.float32)
    check(lib().tpt_debug_hot_kat(device, op, len(a), _ptr(a), _ptr(out)))
    return out


class BVH:
    """BVH (bvh.cuh:60-68): BVH(size) + construct(vertices, indices) -> m_nodes, m_keys.
    Construction runs on the device (src/bvh.cu:304-331 semantics)."""

    def __init__(self, size: int = 0):
        self.size = size
        self.m_nodes = np.zeros(max(2 * size - 1, 0), NODE_DTYPE)
        self.m_keys = np.zeros(size, np.int64)

    def construct(self, device_scene: DeviceScene):
        if not device_scene.built:
            device_scene.build()
        self.m_nodes, self.m_keys = device_scene.read_bvh()
        self.size = len(self.m_keys)
        return self


def procedural_sky(width=2048, height=1024):
    """Deterministic equirect RGBA8 stand-in for the missing kloppenheim env
    (SURVEY 8(d) C3).  Returns rows top-down (image order)."""
    v = (np.arange(height, dtype=np.float64) + 0.5) / height          # 0 = top
    u = (np.arange(width, dtype=np.float64) + 0.5) / width
    theta = v * np.pi
    phi = u * 2.0 * np.pi
    elev = np.cos(theta)[:, None]
    sky = np.clip(elev, 0.0, 1.0)
    ground = np.clip(-elev, 0.0, 1.0)
    sun = np.exp(-((theta[:, None] - 0.9) ** 2 + (np.cos(phi[None, :]) - 1.0) ** 2) * 40.0)
    r = 0.45 + 0.25 * sky - 0.25 * ground + 0.5 * sun
    g = 0.55 + 0.25 * sky - 0.30 * ground + 0.45 * sun
    b = 0.75 + 0.20 * sky - 0.45 * ground + 0.30 * sun
    img = np.stack([r + 0 * phi[None, :], g + 0 * phi[None, :], b + 0 * phi[None, :]], -1)
    img = np.clip(img * 255.0, 0, 255).astype(np.uint8)
    alpha = np.full((height, width, 1), 255, np.uint8)
    return np.concatenate([img, alpha], -1)


class EnvLight:
    """EnvLight (env_light.cuh:8-18): equirect radiance, used on miss (A14).
    Accepts an image file or an RGBA/RGB array in image order (row 0 = top);
    stored row 0 = bottom like FreeImage (picture.h:41-43).  JPEG and binary
    PPM files are decoded by the library's native decoder (tpt_env_load, the
    FreeImage/libjpeg arithmetic); other formats go through PIL."""

    def __init__(self, source=None, device: int = 0):
        self.device = device
        self.handle = C.c_void_p()
        if source is None or (isinstance(source, str) and source == ""):
            self.rgba = None
            return
        if isinstance(source, str):
            if self._native(source):
                self.rgba = None
                check(lib().tpt_env_load(source.encode(), device, C.byref(self.handle)))
                return
            img = self._read(source)
        else:
            img = np.asarray(source, np.uint8)
        if img.ndim != 3 or img.shape[2] not in (3, 4):
            raise RuntimeError("Failed to create texture! Choose picture with 3 or 4 channels.")
        if img.shape[2] == 3:
            img = np.concatenate([img, np.full(img.shape[:2] + (1,), 255, np.uint8)], -1)
        self.rgba = np.ascontiguousarray(img[::-1])           # bottom-up
        h, w = self.rgba.shape[:2]
        check(lib().tpt_env_create(_ptr(self.rgba), w, h, device, C.byref(self.handle)))

    @staticmethod
    def _native(path):
        try:
            with open(path, "rb") as f:
                head = f.read(2)
        except OSError as e:
            raise RuntimeError(f"Failed to open file {path}") from e
        return head in (b"\xff\xd8", b"P6")

    @staticmethod
    def _read(path):
        try:
            from PIL import Image
        except ImportError as e:   # pragma: no cover
            raise RuntimeError(f"Failed to open file {path}: no image decoder") from e
        try:
            with Image.open(path) as im:
                return np.asarray(im.convert("RGBA"))
        except OSError as e:
            raise RuntimeError(f"Failed to open file {path}") from e

    def close(self):
        if self.handle:
            lib().tpt_env_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class Frame:
    bgra: np.ndarray            # [H, W, 4] uint8, row 0 = top (copyToFB layout)
    radiance: np.ndarray        # [H, W, 3] float32, row 0 = bottom (color / spp)
    stats: dict = field(default_factory=dict)


class PathTracer:
    """PathTracer (include/path_tracer.h:16-35), headless.

    The reference renders into a 1920x1080 Vulkan window forever, reseeding the
    RNG with time() and drawing 64 spp per frame (path_tracer.cu:556-579).  Here
    render() draws `frames` frames and returns the last one; seed=None keeps the
    reference's time() seeding, an integer makes the frame reproducible."""

    def __init__(self, envLightFile: str = "", width: int = 1920, height: int = 1080, device: int = 0):
        self.m_width, self.m_height, self.device = width, height, device
        self.envLight = EnvLight(envLightFile, device) if envLightFile else None

    def doTrace(self, d_scene: DeviceScene, camera: Camera, framebuffer=None, nSamplesPerPixel: int = 64,
                seed=None, max_depth: int = 8, radiance=None, band=(16, 1, 0), spp_per_launch: int = 0,
                flags: int = 0, refill: int = 0, accumulate: bool = False, pipe_sets: int = 0,
                pipe_chunks: int = 0, lanes_per_pixel: int = 0, leaf_batch: int = 0, wf_slots: int = 0,
                wf_refill: int = 0, band_list=None, band_cost=None):
        """One frame (path_tracer.cu:491-554).  framebuffer/radiance: numpy (host)
        or torch CUDA tensors / raw device pointers (device, int).
        accumulate=True: progressive rendering (TPT_FLAG_ACCUMULATE) -- continue
        the previous call's samples of the same frame; with seed None the
        previous seed is kept (the reference re-seeds from time() every frame).
        band = (band_rows, band_count, band_index): the interleaved deal;
        band_list: an explicit deal (ascending global band ids of band_rows
        rows each; band_count/band_index ignored); band_cost: a float32 array of
        ceil(H / band_rows) entries that receives the rendered bands' costs
        (tpt_params.band_cost, shard.cost_deal)."""
        if not d_scene.built:
            d_scene.build()
        W, H = self.m_width, self.m_height
        if accumulate:
            flags |= _lib.FLAG_ACCUMULATE
            if seed is None:
                seed = getattr(self, "_last_seed", None)
        if seed is None:
            seed = int(time.time())
        self._last_seed = seed
        p = _lib.Params(W, H, nSamplesPerPixel, max_depth, seed, band[0], band[1], band[2], spp_per_launch,
                        flags | _forced_flags(), refill, pipe_sets, pipe_chunks, lanes_per_pixel, leaf_batch, wf_slots,
                        wf_refill)
        keep = _deal_params(p, H, band, band_list, band_cost)  # noqa: F841 (alive through the call)
        st = _lib.Stats()
        env = self.envLight.handle if self.envLight is not None else None
        rad_p = _addr(radiance)
        fb_p = _addr(framebuffer)
        cam = camera.to_c()
        check(lib().tpt_render(d_scene.handle, env, C.byref(cam), C.byref(p), rad_p, fb_p, C.byref(st)))
        return st.as_dict()

    def doTraceFrames(self, d_scene: DeviceScene, camera: Camera, seeds, framebuffers=None,
                      nSamplesPerPixel: int = 64, max_depth: int = 8, radiances=None, band=(16, 1, 0),
                      spp_per_launch: int = 0, flags: int = 0, refill: int = 0, accumulate: bool = False,
                      pipe_sets: int = 0, pipe_chunks: int = 0, lanes_per_pixel: int = 0, leaf_batch: int = 0,
                      wf_slots: int = 0, wf_refill: int = 0, band_list=None, band_cost=None):
        """A batch of independent frames in one trace launch (tpt_render_frames):
        frame f is doTrace(..., seed=seeds[f]) bit for bit.  framebuffers /
        radiances: None or one buffer (or None) per frame.  band / band_list /
        band_cost as in doTrace."""
        if not d_scene.built:
            d_scene.build()
        seeds = [int(x) for x in seeds]
        n = len(seeds)
        if n == 0:
            raise ValueError("no frames")
        if accumulate:
            flags |= _lib.FLAG_ACCUMULATE
        W, H = self.m_width, self.m_height
        p = _lib.Params(W, H, nSamplesPerPixel, max_depth, seeds[0], band[0], band[1], band[2], spp_per_launch,
                        flags | _forced_flags(), refill, pipe_sets, pipe_chunks, lanes_per_pixel, leaf_batch, wf_slots,
                        wf_refill)
        keep = _deal_params(p, H, band, band_list, band_cost)  # noqa: F841
        st = _lib.Stats()
        env = self.envLight.handle if self.envLight is not None else None

        def ptrs(bufs):
            if bufs is None:
                return None
            if len(bufs) != n:
                raise ValueError("need one output buffer per frame")
            arr = (C.c_void_p * n)(*[(_addr(b).value if b is not None else None) for b in bufs])
            return C.cast(arr, C.POINTER(C.c_void_p)), arr

        rp, fp = ptrs(radiances), ptrs(framebuffers)
        cs = (C.c_uint64 * n)(*seeds)
        cam = camera.to_c()
        check(lib().tpt_render_frames(d_scene.handle, env, C.byref(cam), C.byref(p), n, cs,
                                      rp[0] if rp else None, fp[0] if fp else None, C.byref(st)))
        return st.as_dict()

    def render(self, meshFile: str, nSamplesPerPixel: int = 64, seed=None, max_depth: int = 8, frames: int = 1):
        scene = Scene(meshFile, "gltf")
        d_scene = scene.copySceneToDevice(self.device).build()
        fb = np.zeros((self.m_height, self.m_width, 4), np.uint8)
        fb[..., 3] = 255
        rad = np.zeros((self.m_height, self.m_width, 3), np.float32)
        stats = {}
        for _ in range(frames):
            stats = self.doTrace(d_scene, scene.m_camera, fb, nSamplesPerPixel, seed, max_depth, rad)
        d_scene.close()
        return Frame(fb, rad, stats)


# Test hook: OR-ed into every render's flags, so a whole parity suite can run
# through a variant.  Only tests/conftest.py sets it (from TPT_TEST_FORCE_FLAGS,
# e.g. 32 = TPT_FLAG_WAVEFRONT); the library itself reads no environment.
test_force_flags = 0


def _forced_flags() -> int:
    return int(test_force_flags)


def _deal_params(p, height, band, band_list, band_cost):
    """Fill tpt_params' explicit deal / cost output; returns the ctypes buffers
    that must stay alive through the call."""
    keep = []
    if band_list is not None:
        arr = (C.c_int32 * max(len(band_list), 1))(*[int(b) for b in band_list])
        p.band_list_len = len(band_list)
        p.band_list = C.cast(arr, C.POINTER(C.c_int32))
        keep.append(arr)
    if band_cost is not None:
        nb = (height + band[0] - 1) // band[0]
        if not (isinstance(band_cost, np.ndarray) and band_cost.dtype == np.float32 and band_cost.size == nb
                and band_cost.flags["C_CONTIGUOUS"]):
            raise ValueError(f"band_cost: a contiguous float32 array of {nb} entries")
        p.band_cost = band_cost.ctypes.data_as(C.POINTER(C.c_float))
        keep.append(band_cost)
    return keep


def _addr(buf):
    if buf is None:
        return None
    if isinstance(buf, int):
        return C.c_void_p(buf)
    if isinstance(buf, np.ndarray):
        if not buf.flags["C_CONTIGUOUS"]:
            raise ValueError("output buffers must be contiguous")
        return C.c_void_p(buf.ctypes.data)
    if hasattr(buf, "data_ptr"):             # torch tensor (device memory)
        if not buf.is_contiguous():
            raise ValueError("output tensors must be contiguous")
        if getattr(buf, "is_cuda", False):
            # the library writes device outputs on its own stream (tpt.h): work the
            # caller queued on torch's stream (allocation fill, earlier reads) must be
            # done first
            import torch
            torch.cuda.current_stream(buf.device).synchronize()
        return C.c_void_p(buf.data_ptr())
    raise TypeError(f"unsupported buffer type {type(buf)}")
