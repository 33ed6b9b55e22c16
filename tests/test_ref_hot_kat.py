"""Known-answer tests for the hot path's device functions, pinned to the
reference's OWN headers (tests/golden/ref_hot_kat.json, written by
tests/golden/make_golden.py from oracle/_ref/ref_hot_kat: include/
geometry_queries.h:18-86, delta_light.h:25-130 and material.h:74-103
compiled here by hipcc, host only, no stand-in headers).

* CPU: the oracle's rayHitBBox / rayHitTriangle / DeltaLight::sample /
  CalcDistAttenuation / toUChar / Material() restatements reproduce every
  known answer bit for bit -- the oracle's hot-path arithmetic is pinned to
  the reference, not only to itself.
* GPU: the trace kernel's own device functions (box_hit, the min/max slab
  form, tri_core, light_sample, to_uchar; tpt_debug_hot_kat) reproduce the
  same answers bit for bit.  The min/max slab form is the kernel's fast path
  only for rays whose six slab products are not NaN (finite origin, 1/dir and
  box); it is checked on exactly those cases.

NaN outputs are compared as "both NaN": x86 and the GPU produce different
default-NaN bit patterns for invalid operations (0/0, 0*inf).
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden", "ref_hot_kat.json")


def _f(h):
    return np.frombuffer(bytes.fromhex(h)[::-1], np.float32)[0]


def _bits(x):
    return int(np.frombuffer(np.float32(x).tobytes(), np.uint32)[0])


def same(a, b):
    a, b = np.float32(a), np.float32(b)
    return (np.isnan(a) and np.isnan(b)) or _bits(a) == _bits(b)


@pytest.fixture(scope="module")
def kat():
    with open(GOLD) as f:
        return json.load(f)["kat"]


def _rows(kat, op):
    rows = []
    for e in kat[op]:
        ins = e["in"]
        if op == "L":
            ins = [float(int(ins[0]))] + [_f(h) for h in ins[1:]]
        else:
            ins = [_f(h) for h in ins]
        rows.append((np.array(ins, np.float32), e["out"]))
    return rows


def _fa(v):
    return (C.c_float * len(v))(*[float(x) for x in v])


def test_fixture_covers_the_edge_cases(kat):
    b = _rows(kat, "B")
    x = _rows(kat, "X")
    assert len(b) >= 800 and len(x) >= 600 and len(kat["L"]) >= 120 and len(kat["U"]) >= 60
    d = np.array([r[0][3:6] for r in b])
    assert np.isnan(d).any() and np.isinf(d).any() and (d == 0).any()
    assert any(o[0] == "1" for _, o in b) and any(o[0] == "0" for _, o in b)
    # triangle: both verdicts, negative dist, dist below Delta
    hits = [(r, o) for r, o in x if o[0] == "1"]
    assert len(hits) > 100 and len(hits) < len(x)
    dist = np.array([_f(o[1]) for _, o in hits])
    assert (dist < 0).any() and ((dist > 0) & (dist < 2e-4)).any()


def test_oracle_box_hit_matches_reference(kat):
    L = O.lib()
    L.orc_kat_box_hit.restype = C.c_int
    for r, out in _rows(kat, "B"):
        got = L.orc_kat_box_hit(_fa(r[0:3]), _fa(r[3:6]), _fa(r[6:9]), _fa(r[9:12]))
        assert got == int(out[0]), (r, out)


def test_oracle_triangle_matches_reference(kat):
    L = O.lib()
    L.orc_kat_tri.restype = C.c_int
    for r, out in _rows(kat, "X"):
        o3 = (C.c_float * 3)()
        hit = L.orc_kat_tri(_fa(r[0:3]), _fa(r[3:6]), _fa(r[6:9]), _fa(r[9:12]), _fa(r[12:15]), o3)
        assert hit == int(out[0]), (r, out)
        if hit:
            assert all(same(o3[k], _f(out[1 + k])) for k in range(3)), (r, out, list(o3))


def test_oracle_light_sample_matches_reference(kat):
    L = O.lib()
    for r, out in _rows(kat, "L"):
        lt = O.Light(int(r[0]), (C.c_float * 3)(*r[1:4]), float(r[4]), (C.c_float * 3)(*r[5:8]),
                     (C.c_float * 3)(*r[8:11]), float(r[11]), float(r[12]))
        d3, r3 = (C.c_float * 3)(), (C.c_float * 3)()
        L.orc_kat_light(C.byref(lt), _fa(r[13:16]), d3, r3)
        ref_rad, ref_dir = [_f(h) for h in out[0:3]], [_f(h) for h in out[3:6]]
        assert all(same(r3[k], ref_rad[k]) for k in range(3)), (r, out, list(r3))
        assert all(same(d3[k], ref_dir[k]) for k in range(3)), (r, out, list(d3))


def test_oracle_dist_attenuation_matches_reference(kat):
    L = O.lib()
    L.orc_kat_dist_atten.argtypes = [C.c_float, C.POINTER(C.c_float)]
    for r, out in _rows(kat, "A"):
        rgb = _fa(r[1:4])
        L.orc_kat_dist_atten(float(r[0]), rgb)
        assert all(same(rgb[k], _f(out[k])) for k in range(3)), (r, out, list(rgb))


def test_oracle_to_uchar_and_material_match_reference(kat):
    L = O.lib()
    for r, out in _rows(kat, "U"):
        b = (C.c_uint8 * 3)()
        L.orc_kat_to_uchar(_fa(r), b)
        assert list(b) == [int(v) for v in out], (r, out)
    m = O.Material()
    L.orc_kat_default_material(C.byref(m))
    assert ["%08x" % _bits(v) for v in m.v] == kat["M"][0]["out"]


# ---------------------------------------------------------------------------
# GPU: the trace kernel's own device functions
# ---------------------------------------------------------------------------

@pytest.mark.gpu
def test_kernel_box_tests_match_reference(kat, gpu_available):
    import tinypathtracer_amd as T
    rows = _rows(kat, "B")
    a = np.stack([r for r, _ in rows])
    got = T.hot_kat(0, a)
    ref = np.array([int(o[0]) for _, o in rows])
    assert np.array_equal(got[:, 0].astype(int), ref)           # box_hit: every case
    o, d, lo, hi = a[:, 0:3], a[:, 3:6], a[:, 6:9], a[:, 9:12]
    with np.errstate(all="ignore"):
        inv = (np.float32(1.0) / d).astype(np.float32)
        prods = np.concatenate([(lo - o) * inv, (hi - o) * inv], 1)
    fast = ~np.isnan(prods).any(1) & np.isfinite(o).all(1) & np.isfinite(inv).all(1)
    assert fast.sum() > 300
    assert np.array_equal(got[fast, 1].astype(int), ref[fast])   # min/max form where the kernel uses it


@pytest.mark.gpu
def test_kernel_triangle_matches_reference(kat, gpu_available):
    import tinypathtracer_amd as T
    rows = _rows(kat, "X")
    got = T.hot_kat(1, np.stack([r for r, _ in rows]))
    for (r, out), g in zip(rows, got):
        assert int(g[0]) == int(out[0]), (r, out, g)
        if int(out[0]):
            assert all(same(g[1 + k], _f(out[1 + k])) for k in range(3)), (r, out, g)


@pytest.mark.gpu
def test_kernel_light_and_bytes_match_reference(kat, gpu_available):
    import tinypathtracer_amd as T
    rows = _rows(kat, "L")
    got = T.hot_kat(2, np.stack([r for r, _ in rows]))
    for (r, out), g in zip(rows, got):
        ref_rad, ref_dir = [_f(h) for h in out[0:3]], [_f(h) for h in out[3:6]]
        assert all(same(g[k], ref_dir[k]) for k in range(3)), (r, out, g)
        assert all(same(g[3 + k], ref_rad[k]) for k in range(3)), (r, out, g)
    rows = _rows(kat, "U")
    got = T.hot_kat(3, np.stack([r for r, _ in rows]))
    assert np.array_equal(got.astype(int), np.array([[int(v) for v in o] for _, o in rows]))


def test_abi_structs_match_reference_layouts(kat):
    """The C-ABI takes the reference's device arrays as they are (tpt.h
    tpt_scene_desc): Material is tpt_material byte for byte, and DeltaLight
    (delta_light.h:96-130) has tpt_light's offsets except that a directional
    light's direction shares pos's bytes (TPT_DESC_DELTALIGHT_LAYOUT).  The
    sizes and offsets come from the reference's own headers compiled here
    (oracle/_ref/ref_hot_kat op S)."""
    from tinypathtracer_amd import _lib
    out = [int(x) for x in kat["S"][0]["out"]]
    dl_size, o_type, pl_col, pl_int, pl_pos, dl_col, dl_int, dl_dir, sl_col, sl_int, sl_pos, sl_dir, sl_cos, sl_inv = \
        out[:14]
    m_size, m_base, m_emit, m_eta, m_metal, m_gloss, vec3, spec = out[14:]
    L = _lib.Light
    assert dl_size == C.sizeof(L) == 52
    assert o_type == L.type.offset
    for col, inten in ((pl_col, pl_int), (dl_col, dl_int), (sl_col, sl_int)):
        assert col == L.color.offset and inten == L.intensity.offset
    assert pl_pos == sl_pos == L.pos.offset
    assert dl_dir == L.pos.offset                 # the union remap the library applies
    assert sl_dir == L.direction.offset
    assert sl_cos == L.cos_outer.offset and sl_inv == L.inv_cos_cone_diff.offset
    M = _lib.Material
    assert m_size == C.sizeof(M) == 60
    assert m_base == M.base_color.offset and m_emit == M.emission_factor.offset
    assert m_eta == M.eta.offset and m_metal == M.metallic.offset and m_gloss == M.clearcoat_gloss.offset
    assert vec3 == 12 and spec == 12              # Vec3 / Spectrum: 3 floats, no padding
