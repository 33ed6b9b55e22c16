"""Synthesized benchmark scenes.

C5 is not a shipped asset: box + box1 + box2 + light together hold 2,058
triangles.  The recipe: load the four scenes, translate box1 by
(-2.5, 0, 0), box2 by (+2.5, 0, 0) and the icosphere by (0, 3.5, 0) so that no
surfaces are coplanar, keep box's camera, and apply three 1->4 midpoint
subdivisions (normals interpolated and renormalised) -> 2,058 * 64 = 131,712
triangles.  The result is written as an embedded .gltf that the native loader
(tpt_gltf_load) and the oracle loader both read.

Definitions this module fixes (the recipe leaves them open):
  * a translation is added to the node's glTF translation (objects are T*R*S,
    transform.h:28-33, with no hierarchy), so it moves the object in world space;
  * material names are prefixed with the source scene ("box1/white"): the
    reference loader keys materials by name (std::map, mesh.cuh:113), and the
    sources reuse names with different values;
  * subdivision runs in each mesh's local space in float32 on unshared vertices:
    a midpoint is (a + b) * 0.5 and its normal (na + nb) * 0.5 / |.|; both are
    symmetric in a and b, so neighbouring triangles produce identical edge
    midpoints and the mesh stays watertight;
  * only primitives[0] of each mesh is used, as the reference does.
Deterministic: numpy float32 arithmetic is IEEE, so every host writes the same
bytes (tests/test_synth.py pins a digest).
"""
from __future__ import annotations

import base64
import hashlib
import json
import os

import numpy as np

_C5_PARTS = (("box", (0.0, 0.0, 0.0)), ("box1", (-2.5, 0.0, 0.0)), ("box2", (2.5, 0.0, 0.0)),
             ("light", (0.0, 3.5, 0.0)))
C5_LEVELS = 3

_DT = {5120: np.int8, 5121: np.uint8, 5122: np.int16, 5123: np.uint16, 5124: np.int32, 5125: np.uint32,
       5126: np.float32}
_NC = {"SCALAR": 1, "VEC2": 2, "VEC3": 3, "VEC4": 4}


def _buffers(g, base_dir):
    out = []
    for b in g.get("buffers", []):
        uri = b.get("uri", "")
        if uri.startswith("data:"):
            out.append(base64.b64decode(uri.split(",", 1)[1]))
        else:
            with open(os.path.join(base_dir, uri), "rb") as f:
                out.append(f.read())
    return out


def _accessor(g, bufs, i):
    acc = g["accessors"][i]
    bv = g["bufferViews"][acc["bufferView"]]
    dt = np.dtype(_DT[acc["componentType"]])
    nc = _NC[acc["type"]]
    off = bv.get("byteOffset", 0) + acc.get("byteOffset", 0)
    a = np.frombuffer(bufs[bv["buffer"]], dtype=dt, count=acc["count"] * nc, offset=off)
    return a.reshape(acc["count"], nc) if nc > 1 else a


def subdivide(pos: np.ndarray, nrm: np.ndarray, tri: np.ndarray):
    """One 1->4 midpoint subdivision on unshared vertices (float32): for T input
    triangles returns positions and normals (12T, 3) and indices (4T, 3)."""
    a, b, c = tri[:, 0], tri[:, 1], tri[:, 2]
    half = np.float32(0.5)

    def mid(p, i, j):
        return (p[i] + p[j]) * half

    def nmid(n, i, j):
        m = (n[i] + n[j]) * half
        ln = np.sqrt((m * m).sum(axis=1, dtype=np.float32), dtype=np.float32)
        ln = np.where(ln > 0, ln, np.float32(1.0)).astype(np.float32)
        return (m / ln[:, None]).astype(np.float32)

    pa, pb, pc = pos[a], pos[b], pos[c]
    na, nb, nc = nrm[a], nrm[b], nrm[c]
    pab, pbc, pca = mid(pos, a, b), mid(pos, b, c), mid(pos, c, a)
    nab, nbc, nca = nmid(nrm, a, b), nmid(nrm, b, c), nmid(nrm, c, a)
    # four children, counter-clockwise order preserved: (a,ab,ca) (ab,b,bc) (ca,bc,c) (ab,bc,ca)
    P = np.stack([pa, pab, pca, pab, pb, pbc, pca, pbc, pc, pab, pbc, pca], axis=1).reshape(-1, 3)
    N = np.stack([na, nab, nca, nab, nb, nbc, nca, nbc, nc, nab, nbc, nca], axis=1).reshape(-1, 3)
    T = np.arange(P.shape[0], dtype=np.uint32).reshape(-1, 3)
    return P.astype(np.float32), N.astype(np.float32), T


def merged_scene(scene_dir: str, levels: int = C5_LEVELS, parts=_C5_PARTS, extras=(), generator=None) -> dict:
    """Build the C5 glTF document (dict with an embedded buffer).

    parts: (scene, shift) -- every mesh node of the scene, translated; extras:
    (tag, scene, node name, translation, rotation, scale) -- one more copy of a
    node's mesh with that TRS (the exactness scenes, exactness_scene below).
    With the defaults the document is C5's, byte for byte."""
    nodes, meshes, materials, accessors, views = [], [], [], [], []
    blob = bytearray()
    mat_ids = {}
    camera = None

    def add_view(arr: np.ndarray, target: int) -> int:
        nonlocal blob
        while len(blob) % 4:
            blob.append(0)
        off = len(blob)
        raw = np.ascontiguousarray(arr).tobytes()
        blob += raw
        views.append({"buffer": 0, "byteOffset": off, "byteLength": len(raw), "target": target})
        return len(views) - 1

    def mesh_of(g, bufs, nd):
        prim = g["meshes"][nd["mesh"]]["primitives"][0]
        pos = np.asarray(_accessor(g, bufs, prim["attributes"]["POSITION"]), np.float32)
        nrm = np.asarray(_accessor(g, bufs, prim["attributes"]["NORMAL"]), np.float32)
        tri = np.asarray(_accessor(g, bufs, prim["indices"]), np.uint32).reshape(-1, 3)
        for _ in range(levels):
            pos, nrm, tri = subdivide(pos, nrm, tri)
        return prim, pos, nrm, tri

    def add_mesh(g, name, prim, pos, nrm, tri, mesh_name):
        mi = prim.get("material")
        prim_out = {"attributes": {}, "indices": None}
        if mi is not None:
            src = g["materials"][mi]
            key = f"{name}/{src.get('name', str(mi))}"
            if key not in mat_ids:
                m = json.loads(json.dumps(src))
                m["name"] = key
                mat_ids[key] = len(materials)
                materials.append(m)
            prim_out["material"] = mat_ids[key]
        lo, hi = pos.min(axis=0), pos.max(axis=0)
        accessors.append({"bufferView": add_view(pos, 34962), "componentType": 5126, "count": len(pos),
                          "type": "VEC3", "min": [float(v) for v in lo], "max": [float(v) for v in hi]})
        prim_out["attributes"]["POSITION"] = len(accessors) - 1
        accessors.append({"bufferView": add_view(nrm, 34962), "componentType": 5126, "count": len(nrm),
                          "type": "VEC3"})
        prim_out["attributes"]["NORMAL"] = len(accessors) - 1
        accessors.append({"bufferView": add_view(tri.reshape(-1), 34963), "componentType": 5125,
                          "count": int(tri.size), "type": "SCALAR"})
        prim_out["indices"] = len(accessors) - 1
        meshes.append({"name": mesh_name, "primitives": [prim_out]})
        return len(meshes) - 1

    loaded = {}

    def load(name):
        if name not in loaded:
            path = os.path.join(scene_dir, name + ".gltf")
            with open(path) as f:
                g = json.load(f)
            loaded[name] = (g, _buffers(g, os.path.dirname(path)))
        return loaded[name]

    for name, shift in parts:
        g, bufs = load(name)
        for nd in g.get("nodes", []):
            if "camera" in nd:
                if name == "box" and camera is None:
                    camera = (dict(nd), g["cameras"][nd["camera"]])
                continue
            if "mesh" not in nd:
                continue
            prim, pos, nrm, tri = mesh_of(g, bufs, nd)
            mid = add_mesh(g, name, prim, pos, nrm, tri, f"{name}/{nd.get('name', '')}")
            node = {k: v for k, v in nd.items() if k in ("rotation", "scale", "translation")}
            t = [float(v) for v in nd.get("translation", [0.0, 0.0, 0.0])]
            node["translation"] = [float(np.float32(t[i]) + np.float32(shift[i])) for i in range(3)]
            node["name"] = f"{name}/{nd.get('name', '')}"
            node["mesh"] = mid
            nodes.append(node)
    for tag, name, node_name, tr, rot, sc in extras:
        g, bufs = load(name)
        nd = next(n for n in g["nodes"] if n.get("name") == node_name and "mesh" in n)
        prim, pos, nrm, tri = mesh_of(g, bufs, nd)
        mid = add_mesh(g, name, prim, pos, nrm, tri, f"{tag}/{node_name}")
        nodes.append({"name": f"{tag}/{node_name}", "mesh": mid, "translation": [float(v) for v in tr],
                      "rotation": [float(v) for v in rot], "scale": [float(v) for v in sc]})
    cam_node, cam = camera
    cam_node = {k: v for k, v in cam_node.items() if k in ("rotation", "scale", "translation", "name")}
    cam_node["camera"] = 0
    nodes.insert(0, cam_node)
    doc = {
        "asset": {"version": "2.0", "generator": generator or "tinypathtracer_amd.synth (SURVEY 8(d) C5)"},
        "extensionsUsed": ["KHR_materials_emissive_strength", "KHR_materials_transmission", "KHR_materials_ior"],
        "scene": 0,
        "scenes": [{"name": "C5", "nodes": list(range(len(nodes)))}],
        "nodes": nodes, "cameras": [cam], "meshes": meshes, "materials": materials,
        "accessors": accessors, "bufferViews": views,
        "buffers": [{"byteLength": len(blob),
                     "uri": "data:application/octet-stream;base64," + base64.b64encode(bytes(blob)).decode()}],
    }
    return doc


# Exactness scenes (DESIGN.md section 4 "Culling", verdict r04 item 7): content
# the culled traversal's guards were not tuned on, run through the
# TPT_VERIFY_CULL build (tools/gpu_verify.sh).
#   x1s<seed>: box, plus 12 more copies of its two spheres, box2's two cubes and
#     light's icosphere under random rotations (uniform quaternions), non-uniform
#     scales 0.15-0.6 and positions inside the box: arbitrary orientations and
#     interpenetrating closed meshes (one 1->4 subdivision);
#   x2: box, box1 and box2 stacked at the same place (shift 0), one subdivision:
#     every wall duplicated exactly -- runs of equal Morton keys, which the
#     reference's computeNodeRange (bvh.cu:150-217) splits into a node claimed by
#     two parents (a cycle): tpt_scene_build refuses it (build.hip
#     kMaxLbvhDepth), as the oracle does; a test of that refusal;
#   x3: box, box1 behind it (0, 0, -2) and box2 across both (0.7, 0, -2), one
#     subdivision: walls coplanar with their neighbours' (shared edges) and
#     coplanar overlapping walls of different triangulations and materials --
#     exact t ties decided by the leaf-position tie rule, shared-edge hits.
_X1_OBJECTS = (("box", "ball1"), ("box", "ball2"), ("box2", "Cube"), ("box2", "Cube.001"), ("light", "Icosphere"))


def exactness_scene(kind: str, scene_dir: str) -> dict:
    if kind.startswith("x1s"):
        rng = np.random.default_rng(int(kind[3:]))
        extras = []
        for i in range(12):
            sc_name, nd_name = _X1_OBJECTS[i % len(_X1_OBJECTS)]
            q = rng.normal(size=4)
            q /= np.linalg.norm(q)
            base = 0.15 if sc_name == "light" else 0.6   # the icosphere is 1 unit across
            s3 = rng.uniform(0.25, 1.0, 3) * base
            t = rng.uniform([-0.75, 0.15, -0.75], [0.75, 1.85, 0.75])
            extras.append((f"x{i}", sc_name, nd_name, t, q, s3))
        return merged_scene(scene_dir, 1, parts=(("box", (0.0, 0.0, 0.0)),), extras=extras,
                            generator=f"tinypathtracer_amd.synth exactness scene {kind}")
    if kind == "x2":
        z = (0.0, 0.0, 0.0)
        return merged_scene(scene_dir, 1, parts=(("box", z), ("box1", z), ("box2", z)),
                            generator="tinypathtracer_amd.synth exactness scene x2")
    if kind == "x3":
        return merged_scene(scene_dir, 1, parts=(("box", (0.0, 0.0, 0.0)), ("box1", (0.0, 0.0, -2.0)),
                                                 ("box2", (0.7, 0.0, -2.0))),
                            generator="tinypathtracer_amd.synth exactness scene x3")
    raise ValueError(kind)


def write_scene(doc: dict, out_path: str) -> str:
    """Write a glTF document (skipped when an identical file exists). Returns its sha256."""
    text = json.dumps(doc, separators=(",", ":"))
    digest = hashlib.sha256(text.encode()).hexdigest()
    if os.path.exists(out_path):
        with open(out_path, "rb") as f:
            if hashlib.sha256(f.read()).hexdigest() == digest:
                return digest
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    tmp = f"{out_path}.{os.getpid()}.tmp"   # ranks may generate concurrently
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, out_path)
    return digest


def write_c5(out_path: str, scene_dir: str, levels: int = C5_LEVELS) -> str:
    """Write the C5 scene to out_path (skipped when an identical file exists). Returns its sha256."""
    text = json.dumps(merged_scene(scene_dir, levels), separators=(",", ":"))
    digest = hashlib.sha256(text.encode()).hexdigest()
    if os.path.exists(out_path):
        with open(out_path, "rb") as f:
            if hashlib.sha256(f.read()).hexdigest() == digest:
                return digest
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    tmp = f"{out_path}.{os.getpid()}.tmp"   # ranks may generate concurrently
    with open(tmp, "w") as f:
        f.write(text)
    os.replace(tmp, out_path)
    return digest
