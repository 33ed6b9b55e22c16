"""Oracle restatement of the reference scene loader -- TEST INFRASTRUCTURE ONLY.

Restates ``Scene::readFromGLTF`` (src/mesh.cu:80-307) and
``Scene::copySceneToDevice`` (src/mesh.cu:309-397) plus the host math they
use (include/transform.h:16-33, include/math/quat.h:52-69,
include/math/mat.h:17-51, 203-282) in float32, operation for operation, so
the packed arrays are bit-identical to what the reference uploads.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module; the product loader is tinypathtracer_amd/csrc/host/gltf.cpp.
"""
from __future__ import annotations

import base64
import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

F = np.float32


def f32(x) -> np.float32:
    return np.float32(x)


# --------------------------------------------------------------------------
# Mat4 (column-major list of 4 columns, each a list of 4 float32)
# --------------------------------------------------------------------------
def mat_identity():
    return [[F(1) if i == j else F(0) for i in range(4)] for j in range(4)]


def mat_mul(lhs, rhs):
    """MatrixMultiply (mat.h:17-35): res[j][i] += lhs[k][i] * rhs[j][k]."""
    res = [[F(0)] * 4 for _ in range(4)]
    for i in range(4):
        for j in range(4):
            acc = F(0)
            for k in range(4):
                acc = F(acc + F(lhs[k][i] * rhs[j][k]))
            res[j][i] = acc
    return res


def mat_vec(m, v):
    """MatrixVectorMultiply (mat.h:37-51)."""
    out = []
    for i in range(4):
        acc = F(0)
        for j in range(4):
            acc = F(acc + F(m[j][i] * v[j]))
        out.append(acc)
    return out


def mat_transpose(m):
    return [[m[i][j] for i in range(4)] for j in range(4)]


def _prod3(a, b, c):
    return F(F(a * b) * c)


def mat_determinant(c):
    """Mat4::determinant (mat.h:203-228), 24 signed triple products left to right."""
    terms = [
        (+1, (0, 3), (1, 2), (2, 1), (3, 0)), (-1, (0, 2), (1, 3), (2, 1), (3, 0)),
        (-1, (0, 3), (1, 1), (2, 2), (3, 0)), (+1, (0, 1), (1, 3), (2, 2), (3, 0)),
        (+1, (0, 2), (1, 1), (2, 3), (3, 0)), (-1, (0, 1), (1, 2), (2, 3), (3, 0)),
        (-1, (0, 3), (1, 2), (2, 0), (3, 1)), (+1, (0, 2), (1, 3), (2, 0), (3, 1)),
        (+1, (0, 3), (1, 0), (2, 2), (3, 1)), (-1, (0, 0), (1, 3), (2, 2), (3, 1)),
        (-1, (0, 2), (1, 0), (2, 3), (3, 1)), (+1, (0, 0), (1, 2), (2, 3), (3, 1)),
        (+1, (0, 3), (1, 1), (2, 0), (3, 2)), (-1, (0, 1), (1, 3), (2, 0), (3, 2)),
        (-1, (0, 3), (1, 0), (2, 1), (3, 2)), (+1, (0, 0), (1, 3), (2, 1), (3, 2)),
        (+1, (0, 1), (1, 0), (2, 3), (3, 2)), (-1, (0, 0), (1, 1), (2, 3), (3, 2)),
        (-1, (0, 2), (1, 1), (2, 0), (3, 3)), (+1, (0, 1), (1, 2), (2, 0), (3, 3)),
        (+1, (0, 2), (1, 0), (2, 1), (3, 3)), (-1, (0, 0), (1, 2), (2, 1), (3, 3)),
        (-1, (0, 1), (1, 0), (2, 2), (3, 3)), (+1, (0, 0), (1, 1), (2, 2), (3, 3)),
    ]
    acc = None
    for sgn, a, b, cc, d in terms:
        p = F(F(F(c[a[0]][a[1]] * c[b[0]][b[1]]) * c[cc[0]][cc[1]]) * c[d[0]][d[1]])
        if acc is None:
            acc = p if sgn > 0 else F(-p)
        else:
            acc = F(acc + p) if sgn > 0 else F(acc - p)
    return acc


# Mat4::inverse (mat.h:229-282): each r[col][row] is six signed triple products.
# Each entry: list of (sign, (c,r), (c,r), (c,r)) evaluated left to right.
_INV_TERMS = {
    (0, 0): [(+1, (1, 2), (2, 3), (3, 1)), (-1, (1, 3), (2, 2), (3, 1)), (+1, (1, 3), (2, 1), (3, 2)),
             (-1, (1, 1), (2, 3), (3, 2)), (-1, (1, 2), (2, 1), (3, 3)), (+1, (1, 1), (2, 2), (3, 3))],
    (0, 1): [(+1, (0, 3), (2, 2), (3, 1)), (-1, (0, 2), (2, 3), (3, 1)), (-1, (0, 3), (2, 1), (3, 2)),
             (+1, (0, 1), (2, 3), (3, 2)), (+1, (0, 2), (2, 1), (3, 3)), (-1, (0, 1), (2, 2), (3, 3))],
    (0, 2): [(+1, (0, 2), (1, 3), (3, 1)), (-1, (0, 3), (1, 2), (3, 1)), (+1, (0, 3), (1, 1), (3, 2)),
             (-1, (0, 1), (1, 3), (3, 2)), (-1, (0, 2), (1, 1), (3, 3)), (+1, (0, 1), (1, 2), (3, 3))],
    (0, 3): [(+1, (0, 3), (1, 2), (2, 1)), (-1, (0, 2), (1, 3), (2, 1)), (-1, (0, 3), (1, 1), (2, 2)),
             (+1, (0, 1), (1, 3), (2, 2)), (+1, (0, 2), (1, 1), (2, 3)), (-1, (0, 1), (1, 2), (2, 3))],
    (1, 0): [(+1, (1, 3), (2, 2), (3, 0)), (-1, (1, 2), (2, 3), (3, 0)), (-1, (1, 3), (2, 0), (3, 2)),
             (+1, (1, 0), (2, 3), (3, 2)), (+1, (1, 2), (2, 0), (3, 3)), (-1, (1, 0), (2, 2), (3, 3))],
    (1, 1): [(+1, (0, 2), (2, 3), (3, 0)), (-1, (0, 3), (2, 2), (3, 0)), (+1, (0, 3), (2, 0), (3, 2)),
             (-1, (0, 0), (2, 3), (3, 2)), (-1, (0, 2), (2, 0), (3, 3)), (+1, (0, 0), (2, 2), (3, 3))],
    (1, 2): [(+1, (0, 3), (1, 2), (3, 0)), (-1, (0, 2), (1, 3), (3, 0)), (-1, (0, 3), (1, 0), (3, 2)),
             (+1, (0, 0), (1, 3), (3, 2)), (+1, (0, 2), (1, 0), (3, 3)), (-1, (0, 0), (1, 2), (3, 3))],
    (1, 3): [(+1, (0, 2), (1, 3), (2, 0)), (-1, (0, 3), (1, 2), (2, 0)), (+1, (0, 3), (1, 0), (2, 2)),
             (-1, (0, 0), (1, 3), (2, 2)), (-1, (0, 2), (1, 0), (2, 3)), (+1, (0, 0), (1, 2), (2, 3))],
    (2, 0): [(+1, (1, 1), (2, 3), (3, 0)), (-1, (1, 3), (2, 1), (3, 0)), (+1, (1, 3), (2, 0), (3, 1)),
             (-1, (1, 0), (2, 3), (3, 1)), (-1, (1, 1), (2, 0), (3, 3)), (+1, (1, 0), (2, 1), (3, 3))],
    (2, 1): [(+1, (0, 3), (2, 1), (3, 0)), (-1, (0, 1), (2, 3), (3, 0)), (-1, (0, 3), (2, 0), (3, 1)),
             (+1, (0, 0), (2, 3), (3, 1)), (+1, (0, 1), (2, 0), (3, 3)), (-1, (0, 0), (2, 1), (3, 3))],
    (2, 2): [(+1, (0, 1), (1, 3), (3, 0)), (-1, (0, 3), (1, 1), (3, 0)), (+1, (0, 3), (1, 0), (3, 1)),
             (-1, (0, 0), (1, 3), (3, 1)), (-1, (0, 1), (1, 0), (3, 3)), (+1, (0, 0), (1, 1), (3, 3))],
    (2, 3): [(+1, (0, 3), (1, 1), (2, 0)), (-1, (0, 1), (1, 3), (2, 0)), (-1, (0, 3), (1, 0), (2, 1)),
             (+1, (0, 0), (1, 3), (2, 1)), (+1, (0, 1), (1, 0), (2, 3)), (-1, (0, 0), (1, 1), (2, 3))],
    (3, 0): [(+1, (1, 2), (2, 1), (3, 0)), (-1, (1, 1), (2, 2), (3, 0)), (-1, (1, 2), (2, 0), (3, 1)),
             (+1, (1, 0), (2, 2), (3, 1)), (+1, (1, 1), (2, 0), (3, 2)), (-1, (1, 0), (2, 1), (3, 2))],
    (3, 1): [(+1, (0, 1), (2, 2), (3, 0)), (-1, (0, 2), (2, 1), (3, 0)), (+1, (0, 2), (2, 0), (3, 1)),
             (-1, (0, 0), (2, 2), (3, 1)), (-1, (0, 1), (2, 0), (3, 2)), (+1, (0, 0), (2, 1), (3, 2))],
    (3, 2): [(+1, (0, 2), (1, 1), (3, 0)), (-1, (0, 1), (1, 2), (3, 0)), (-1, (0, 2), (1, 0), (3, 1)),
             (+1, (0, 0), (1, 2), (3, 1)), (+1, (0, 1), (1, 0), (3, 2)), (-1, (0, 0), (1, 1), (3, 2))],
    (3, 3): [(+1, (0, 1), (1, 2), (2, 0)), (-1, (0, 2), (1, 1), (2, 0)), (+1, (0, 2), (1, 0), (2, 1)),
             (-1, (0, 0), (1, 2), (2, 1)), (-1, (0, 1), (1, 0), (2, 2)), (+1, (0, 0), (1, 1), (2, 2))],
}


def mat_inverse(c):
    r = [[F(0)] * 4 for _ in range(4)]
    for (col, row), terms in _INV_TERMS.items():
        acc = None
        for sgn, a, b, d in terms:
            p = _prod3(c[a[0]][a[1]], c[b[0]][b[1]], c[d[0]][d[1]])
            if acc is None:
                acc = p if sgn > 0 else F(-p)
            else:
                acc = F(acc + p) if sgn > 0 else F(acc - p)
        r[col][row] = acc
    s = F(F(1.0) / mat_determinant(c))
    return [[F(r[j][i] * s) for i in range(4)] for j in range(4)]


def rotate_from_quat(w, x, y, z):
    """Quat::RotateFromQuat (quat.h:52-69) -> Mat4 via Mat4(const Mat3&) (mat.h:175)."""
    x2, y2, z2 = F(x * x), F(y * y), F(z * z)
    xy, xz, yz = F(x * y), F(x * z), F(y * z)
    wx, wy, wz = F(w * x), F(w * y), F(w * z)
    two, one = F(2), F(1)
    c0 = [F(one - F(two * F(y2 + z2))), F(two * F(xy + wz)), F(two * F(xz - wy)), F(0)]
    c1 = [F(two * F(xy - wz)), F(one - F(two * F(x2 + z2))), F(two * F(yz + wx)), F(0)]
    c2 = [F(two * F(xz + wy)), F(two * F(yz - wx)), F(one - F(two * F(x2 + y2))), F(0)]
    return [c0, c1, c2, [F(0), F(0), F(0), F(1)]]


def local_to_world(loc, quat_wxyz, scale):
    """Transform::localToParent (transform.h:28-33): (T * R) * S."""
    t = mat_identity()
    t[3] = [F(loc[0]), F(loc[1]), F(loc[2]), F(1)]
    r = rotate_from_quat(*quat_wxyz)
    s = mat_identity()
    s[0][0], s[1][1], s[2][2] = F(scale[0]), F(scale[1]), F(scale[2])
    return mat_mul(mat_mul(t, r), s)


def normal_to_world(l2w):
    """copySceneToDevice's normal_to_world lambda (mesh.cu:370-378)."""
    m = [[l2w[0][0], l2w[0][1], l2w[0][2], F(0)],
         [l2w[1][0], l2w[1][1], l2w[1][2], F(0)],
         [l2w[2][0], l2w[2][1], l2w[2][2], F(0)],
         [F(0), F(0), F(0), F(1)]]
    return mat_inverse(mat_transpose(m))


def flat(m):
    return np.array([m[j][i] for j in range(4) for i in range(4)], dtype=np.float32)


# --------------------------------------------------------------------------
# Scene
# --------------------------------------------------------------------------
MATERIAL_DEFAULT = dict(  # Material() (material.h:88-103)
    base_color=(F(0.82), F(0.67), F(0.16)), emission_factor=F(0), eta=F(0), metallic=F(0),
    subsurface=F(0), specular=F(0.5), roughness=F(0.5), specular_tint=F(0), anisotropic=F(0),
    sheen=F(0), sheen_tint=F(0), clearcoat=F(0), clearcoat_gloss=F(1))
MATERIAL_FIELDS = ["base_color", "emission_factor", "eta", "metallic", "subsurface", "specular",
                   "roughness", "specular_tint", "anisotropic", "sheen", "sheen_tint", "clearcoat",
                   "clearcoat_gloss"]

LIGHT_POINT, LIGHT_DIRECTIONAL, LIGHT_SPOT = 0, 1, 2
WATTS_PER_LUMEN = F(F(1.0) / F(683.0))   # delta_light.h:6


@dataclass
class OracleScene:
    indices: np.ndarray          # uint32 [3F]
    vertices: np.ndarray         # float32 [V,3]
    normals: np.ndarray          # float32 [V,3]
    lut: np.ndarray              # int32 [O,2] (begin, mtl)
    vert_trans: np.ndarray       # float32 [O,16]
    normal_trans: np.ndarray     # float32 [O,16]
    materials: np.ndarray        # float32 [M,15]
    material_names: list
    lights: list                 # dicts
    camera_c2w: np.ndarray       # float32 [16]
    vfov: np.float32
    aspect: np.float32
    znear: np.float32
    missing_material: bool = False
    meta: dict = field(default_factory=dict)

    @property
    def n_faces(self):
        return len(self.indices) // 3


def _accessor_array(model, buffers, acc_idx):
    acc = model["accessors"][acc_idx]
    bv = model["bufferViews"][acc["bufferView"]]
    buf = buffers[bv.get("buffer", 0)]
    off = acc.get("byteOffset", 0) + bv.get("byteOffset", 0)
    ncomp = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4}[acc["type"]]
    dt = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16,
          5124: np.int32, 5125: np.uint32, 5126: np.float32}[acc["componentType"]]
    count = acc["count"]
    return np.frombuffer(buf, dtype=dt, count=count * ncomp, offset=off).reshape(count, ncomp) \
        if ncomp > 1 else np.frombuffer(buf, dtype=dt, count=count, offset=off)


def _decode_buffers(model, base_dir):
    out = []
    for b in model.get("buffers", []):
        uri = b.get("uri", "")
        if uri.startswith("data:"):
            out.append(base64.b64decode(uri.split(",", 1)[1]))
        else:
            with open(os.path.join(base_dir, uri), "rb") as fh:
                out.append(fh.read())
    return out


def _read_transform(node):
    """readTransform lambda (mesh.cu:102-138): Quat() = 0 when absent (App. A.11)."""
    r = node.get("rotation")
    q = (F(r[3]), F(r[0]), F(r[1]), F(r[2])) if r else (F(0), F(0), F(0), F(0))
    s = node.get("scale")
    sc = (F(s[0]), F(s[1]), F(s[2])) if s else (F(1), F(1), F(1))
    t = node.get("translation")
    tr = (F(t[0]), F(t[1]), F(t[2])) if t else (F(0), F(0), F(0))
    return tr, q, sc


def load_gltf(path: str) -> OracleScene:
    with open(path, "rb") as fh:
        model = json.loads(fh.read())
    buffers = _decode_buffers(model, os.path.dirname(path))
    meshes = []
    materials: dict = {}
    lights: dict = {}
    cam = None
    missing_material = False
    for node in model.get("nodes", []):
        if node.get("camera", -1) > -1:
            ci = model["cameras"][node["camera"]]
            if ci.get("type") == "perspective":
                p = ci.get("perspective", {})
                tr, q, sc = _read_transform(node)
                cam = (local_to_world(tr, q, sc), F(p.get("yfov", 0.0)),
                       F(p.get("aspectRatio", 0.0)), F(p.get("znear", 0.0)))
        elif node.get("mesh", -1) > -1:
            mesh = model["meshes"][node["mesh"]]
            prim = mesh["primitives"][0]
            attrs = prim["attributes"]
            pos = _accessor_array(model, buffers, attrs["POSITION"]).astype(np.float32)
            ind = _accessor_array(model, buffers, prim["indices"]).astype(np.int64).astype(np.uint32)
            nrm = _accessor_array(model, buffers, attrs["NORMAL"]).astype(np.float32)
            mname = ""
            if model.get("materials"):
                mi = prim.get("material", -1)
                if mi < 0:
                    missing_material = True   # reference indexes materials[-1] (UB): defined as ""
                else:
                    mat = model["materials"][mi]
                    mname = mat.get("name", "")
                    if mname not in materials:
                        m = dict(MATERIAL_DEFAULT)
                        pbr = mat.get("pbrMetallicRoughness", {})
                        m["roughness"] = F(pbr.get("roughnessFactor", 1.0))
                        m["metallic"] = F(pbr.get("metallicFactor", 1.0))
                        bc = pbr.get("baseColorFactor", [1.0, 1.0, 1.0, 1.0])
                        m["base_color"] = (F(bc[0]), F(bc[1]), F(bc[2]))
                        for key, val in mat.get("extensions", {}).items():
                            if key == "KHR_materials_transmission":
                                m["specular"] = F(F(1.0) - F(F(val["transmissionFactor"]) / F(5.0)))
                            if key == "KHR_materials_emissive_strength":
                                m["emission_factor"] = F(val["emissiveStrength"])
                            if key == "KHR_materials_ior":
                                m["eta"] = F(val["ior"])
                        materials[mname] = m
            else:
                missing_material = True
            tr, q, sc = _read_transform(node)
            meshes.append(dict(pos=pos, ind=ind, nrm=nrm, material=mname, l2w=local_to_world(tr, q, sc)))
        else:
            ext = node.get("extensions", {}).get("KHR_lights_punctual")
            if ext is None:
                continue
            light = model["extensions"]["KHR_lights_punctual"]["lights"][ext["light"]]
            name = node.get("name", "")
            tr, q, sc = _read_transform(node)
            m = local_to_world(tr, q, sc)
            color = [F(c) for c in light.get("color", [1.0, 1.0, 1.0])]
            d = dict(type=0, color=color, intensity=F(0), pos=[F(0)] * 3, direction=[F(0)] * 3,
                     cos_outer=F(0), inv_cos_cone_diff=F(0))
            lt = light.get("type")
            if lt == "point":
                d["type"] = LIGHT_POINT
                d["intensity"] = F(F(light.get("intensity", 1.0)) * WATTS_PER_LUMEN)
                d["pos"] = mat_vec(m, [F(0), F(0), F(0), F(1)])[:3]
            elif lt == "directional":
                d["type"] = LIGHT_DIRECTIONAL
                d["intensity"] = F(light.get("intensity", 1.0))
                d["direction"] = mat_vec(m, [F(0), F(0), F(-1), F(0)])[:3]
            elif lt == "spot":
                d["type"] = LIGHT_SPOT
                d["intensity"] = F(F(light.get("intensity", 1.0)) * WATTS_PER_LUMEN)
                spot = light.get("spot", {})
                inner = F(spot.get("innerConeAngle", 0.0))
                outer = F(spot.get("outerConeAngle", 0.7853981634))
                co = F(math.cos(float(outer)))   # std::cos(float) -- correctly rounded here
                ci = F(math.cos(float(inner)))
                d["cos_outer"] = co
                d["inv_cos_cone_diff"] = F(F(1.0) / F(ci - co))
                d["direction"] = mat_vec(m, [F(0), F(0), F(-1), F(0)])[:3]
                d["pos"] = mat_vec(m, [F(0), F(0), F(0), F(1)])[:3]
            else:
                raise RuntimeError("Unsupported light type")
            lights[name] = d

    # copySceneToDevice (mesh.cu:309-397)
    names = sorted(materials.keys())          # std::map order (byte-wise)
    mat_index = {n: i for i, n in enumerate(names)}
    mats = np.zeros((max(len(names), 0), 15), dtype=np.float32)
    for i, n in enumerate(names):
        m = materials[n]
        row = list(m["base_color"]) + [m[k] for k in MATERIAL_FIELDS[1:]]
        mats[i] = np.array(row, dtype=np.float32)
    idx_all, pos_all, nrm_all, lut, vt, nt = [], [], [], [], [], []
    icount = vcount = 0
    for mesh in meshes:
        idx_all.append(mesh["ind"].astype(np.uint32) + np.uint32(vcount))
        pos_all.append(mesh["pos"])
        nrm_all.append(mesh["nrm"])
        lut.append((icount // 3, mat_index.get(mesh["material"], 0)))
        icount += len(mesh["ind"])
        vcount += len(mesh["pos"])
        vt.append(flat(mesh["l2w"]))
        nt.append(flat(normal_to_world(mesh["l2w"])))
    light_list = [lights[k] for k in sorted(lights.keys())]
    if cam is None:
        c2w, vfov, aspect, znear = flat(mat_identity()), F(60.0), F(1.77778), F(0.1)   # Camera()
    else:
        c2w, vfov, aspect, znear = flat(cam[0]), cam[1], cam[2], cam[3]
    return OracleScene(
        indices=np.concatenate(idx_all).astype(np.uint32),
        vertices=np.concatenate(pos_all).astype(np.float32),
        normals=np.concatenate(nrm_all).astype(np.float32),
        lut=np.array(lut, dtype=np.int32).reshape(-1, 2),
        vert_trans=np.stack(vt).astype(np.float32),
        normal_trans=np.stack(nt).astype(np.float32),
        materials=mats, material_names=names, lights=light_list,
        camera_c2w=c2w, vfov=vfov, aspect=aspect, znear=znear,
        missing_material=missing_material or (len(names) == 0),
    )
