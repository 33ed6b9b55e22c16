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


def merged_scene(scene_dir: str, levels: int = C5_LEVELS) -> dict:
    """Build the C5 glTF document (dict with an embedded buffer)."""
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

    for name, shift in _C5_PARTS:
        path = os.path.join(scene_dir, name + ".gltf")
        with open(path) as f:
            g = json.load(f)
        bufs = _buffers(g, os.path.dirname(path))
        for nd in g.get("nodes", []):
            if "camera" in nd:
                if name == "box" and camera is None:
                    camera = (dict(nd), g["cameras"][nd["camera"]])
                continue
            if "mesh" not in nd:
                continue
            prim = g["meshes"][nd["mesh"]]["primitives"][0]
            pos = np.asarray(_accessor(g, bufs, prim["attributes"]["POSITION"]), np.float32)
            nrm = np.asarray(_accessor(g, bufs, prim["attributes"]["NORMAL"]), np.float32)
            tri = np.asarray(_accessor(g, bufs, prim["indices"]), np.uint32).reshape(-1, 3)
            for _ in range(levels):
                pos, nrm, tri = subdivide(pos, nrm, tri)
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
            meshes.append({"name": f"{name}/{nd.get('name', '')}", "primitives": [prim_out]})
            node = {k: v for k, v in nd.items() if k in ("rotation", "scale", "translation")}
            t = [float(v) for v in nd.get("translation", [0.0, 0.0, 0.0])]
            node["translation"] = [float(np.float32(t[i]) + np.float32(shift[i])) for i in range(3)]
            node["name"] = f"{name}/{nd.get('name', '')}"
            node["mesh"] = len(meshes) - 1
            nodes.append(node)
    cam_node, cam = camera
    cam_node = {k: v for k, v in cam_node.items() if k in ("rotation", "scale", "translation", "name")}
    cam_node["camera"] = 0
    nodes.insert(0, cam_node)
    doc = {
        "asset": {"version": "2.0", "generator": "tinypathtracer_amd.synth (SURVEY 8(d) C5)"},
        "extensionsUsed": ["KHR_materials_emissive_strength", "KHR_materials_transmission", "KHR_materials_ior"],
        "scene": 0,
        "scenes": [{"name": "C5", "nodes": list(range(len(nodes)))}],
        "nodes": nodes, "cameras": [cam], "meshes": meshes, "materials": materials,
        "accessors": accessors, "bufferViews": views,
        "buffers": [{"byteLength": len(blob),
                     "uri": "data:application/octet-stream;base64," + base64.b64encode(bytes(blob)).decode()}],
    }
    return doc


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
