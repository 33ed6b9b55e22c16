"""Parity trig (tinypathtracer_amd/csrc/common/ptrig.hpp) on the CPU.

* fsincos_2pi: the kernel's fp32 sin/cos of phi = 2*pi*u.  The header is
  compiled for the host with g++ (the same source the HIP kernel compiles) and
  must agree bit for bit with the oracle's C restatement (trig_mode 1), and
  stay within 1 ulp of the correctly rounded value over the curand input set.
* datan2 / dacos (env lookup): (float) of the double evaluation must equal
  (float) libm's double atan2/acos.
* env_col_fast / env_row_fast (the lookup's texel indices from fp32 bounds):
  the fp32 atan2/acos stay far inside kEnvTrigBound, and wherever the fast
  indices decide they equal the double path's, on random directions and on
  directions placed at texel edges.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from tests.conftest import ROOT

HARNESS = r'''
#include "ptrig.hpp"
#include <cstdio>
#include <cstdint>
#include <cstring>
extern "C" {
void h_sincos(const float* x, float* s, float* c, int n) { for (int i = 0; i < n; ++i) tpt::fsincos_2pi(x[i], s[i], c[i]); }
void h_atan2(const float* y, const float* x, float* o, int n) { for (int i = 0; i < n; ++i) o[i] = tpt::patan2_fast(y[i], x[i]); }
void h_acos(const float* y, float* o, int n) { for (int i = 0; i < n; ++i) o[i] = tpt::pacos_fast(y[i]); }
void h_fatan2(const float* y, const float* x, float* o, int n) { for (int i = 0; i < n; ++i) o[i] = tpt::fatan2_approx(y[i], x[i]); }
// fast indices (-1: undecided) and the double path's (the kernel's env_lookup_inl fallback)
void h_envidx(const float* x, const float* y, const float* z, int n, int w, int h, int* fc, int* fr, int* dc, int* dr) {
    for (int i = 0; i < n; ++i) {
        fc[i] = tpt::env_col_fast(z[i], x[i], w);
        fr[i] = tpt::env_row_fast(y[i], h);
        float u = tpt::patan2_fast(z[i], x[i]) / (2.0f * tpt::kPi);
        if (u < 0.0f) u += 1.0f;
        const float c = y[i] > 1.0f ? 1.0f : (y[i] < -1.0f ? -1.0f : y[i]);
        const float v = 1.0f - tpt::pacos_fast(c) / tpt::kPi;
        int ix = (int)floorf(u * (float)w), iy = (int)floorf(v * (float)h);
        dc[i] = ix < 0 ? 0 : (ix > w - 1 ? w - 1 : ix);
        dr[i] = iy < 0 ? 0 : (iy > h - 1 ? h - 1 : iy);
    }
}
}
'''


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("ptrig")
    src = d / "h.cpp"
    src.write_text(HARNESS)
    so = d / "libh.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
                           "-I", os.path.join(ROOT, "tinypathtracer_amd", "csrc", "common"), str(src), "-o", str(so)])
    L = C.CDLL(str(so))
    for fn in ("h_sincos", "h_atan2", "h_acos", "h_fatan2", "h_envidx"):
        getattr(L, fn).restype = None
    return L


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _phis(n, seed=1):
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    u = (x.astype(np.float32) * np.float32(2.3283064e-10) + np.float32(2.3283064e-10 / 2.0)).astype(np.float32)
    phi = (np.float32(2.0 * np.float32(3.141592653589793)) * u).astype(np.float32)
    edge = np.array([0.0, 1.4629181e-09, 6.2831855, 1.5707964, 3.1415927, 4.712389, 0.7853982], np.float32)
    return np.concatenate([phi, edge])


def test_sincos_kernel_source_equals_oracle(harness):
    phi = _phis(200_000)
    n = len(phi)
    s = np.zeros(n, np.float32)
    c = np.zeros(n, np.float32)
    harness.h_sincos(_p(phi), _p(s), _p(c), n)
    L = O.lib()
    L.orc_parity_sincos.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
    for i in range(0, n, 97):
        os_, oc_ = C.c_float(), C.c_float()
        L.orc_parity_sincos(float(phi[i]), C.byref(os_), C.byref(oc_))
        assert np.float32(os_.value).view(np.uint32) == s[i].view(np.uint32)
        assert np.float32(oc_.value).view(np.uint32) == c[i].view(np.uint32)


def _ulps(a, b):
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7fffffff), ia)
    ib = np.where(ib < 0, -(ib & 0x7fffffff), ib)
    return np.abs(ia - ib)


def test_sincos_within_one_ulp(harness):
    phi = _phis(1_000_000, seed=2)
    n = len(phi)
    s = np.zeros(n, np.float32)
    c = np.zeros(n, np.float32)
    harness.h_sincos(_p(phi), _p(s), _p(c), n)
    rs = np.sin(phi.astype(np.float64)).astype(np.float32)
    rc = np.cos(phi.astype(np.float64)).astype(np.float32)
    assert _ulps(s, rs).max() <= 1
    assert _ulps(c, rc).max() <= 1
    assert (s == rs).mean() > 0.8 and (c == rc).mean() > 0.75


def test_env_atan2_acos_match_libm_double(harness):
    rng = np.random.default_rng(3)
    v = rng.normal(size=(200_000, 3)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True).astype(np.float32)
    v[::7, 0] = 0.0
    v[::11, 2] = -0.0
    y = np.ascontiguousarray(v[:, 2])
    x = np.ascontiguousarray(v[:, 0])
    n = len(x)
    o = np.zeros(n, np.float32)
    harness.h_atan2(_p(y), _p(x), _p(o), n)
    assert np.array_equal(o.view(np.uint32), np.arctan2(y.astype(np.float64), x.astype(np.float64))
                          .astype(np.float32).view(np.uint32))
    yc = np.ascontiguousarray(np.clip(v[:, 1], -1.0, 1.0))
    harness.h_acos(_p(yc), _p(o), n)
    assert np.array_equal(o.view(np.uint32), np.arccos(yc.astype(np.float64)).astype(np.float32).view(np.uint32))


def _dirs(n, seed):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n, 3)).astype(np.float32)
    v /= np.linalg.norm(v, axis=1, keepdims=True).astype(np.float32)
    v[::13, 0] = 0.0
    v[::17, 2] = -0.0
    v[::19, 1] = 1.0
    v[::23, 1] = -1.0
    return v


def _edge_dirs(w, h, seed):
    """Directions whose (u, v) sit on texel edges (and 1 ulp either side)."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(0, w + 1, max(1, w // 256)):
        phi = 2.0 * np.pi * k / w
        th = rng.uniform(0.05, np.pi - 0.05)
        out.append((np.sin(th) * np.cos(phi), np.cos(th), np.sin(th) * np.sin(phi)))
    for k in range(0, h + 1, max(1, h // 256)):
        th = np.pi * (1.0 - k / h)
        phi = rng.uniform(0, 2 * np.pi)
        out.append((np.sin(th) * np.cos(phi), np.cos(th), np.sin(th) * np.sin(phi)))
    v = np.array(out, np.float32)
    nb = [v]
    for d in (-1, 1, -2, 2):   # neighbouring floats of every component
        nb.append(np.nextafter(v, np.float32(d * np.inf)).astype(np.float32))
    return np.concatenate(nb)


def test_env_fast_trig_error_far_inside_bound(harness):
    v = _dirs(400_000, 5)
    x, z = np.ascontiguousarray(v[:, 0]), np.ascontiguousarray(v[:, 2])
    n = len(x)
    o = np.zeros(n, np.float32)
    harness.h_fatan2(_p(z), _p(x), _p(o), n)
    ref = np.arctan2(z.astype(np.float64), x.astype(np.float64))
    ok = np.maximum(np.abs(x), np.abs(z)) >= 1e-18   # the domain env_col_fast uses it on
    err = np.abs(o.astype(np.float64) - ref)[ok]
    assert err.max() < 4.0e-7, err.max()   # kEnvTrigBound is 4e-6: a 10x margin
    c = np.clip(np.ascontiguousarray(v[:, 1]), -1.0, 1.0).astype(np.float32)
    s = np.sqrt(((np.float32(1) - c) * (np.float32(1) + c)).astype(np.float32)).astype(np.float32)
    harness.h_fatan2(_p(s), _p(c), _p(o), n)
    err = np.abs(o.astype(np.float64) - np.arccos(c.astype(np.float64)))
    assert err.max() < 4.0e-7, err.max()


@pytest.mark.parametrize("w,h", [(2048, 1024), (4096, 2048), (512, 256), (1000, 500), (64, 32), (1, 1)])
def test_env_fast_indices_equal_double_path(harness, w, h):
    v = np.concatenate([_dirs(300_000, 7 + w), _edge_dirs(w, h, 11 + h)])
    x, y, z = (np.ascontiguousarray(v[:, i]) for i in range(3))
    n = len(x)
    fc, fr, dc, dr = (np.zeros(n, np.int32) for _ in range(4))
    harness.h_envidx(_p(x), _p(y), _p(z), n, w, h, _p(fc), _p(fr), _p(dc), _p(dr))
    col, row = fc >= 0, fr >= 0
    assert np.array_equal(fc[col], dc[col]), np.flatnonzero(col & (fc != dc))[:5]
    assert np.array_equal(fr[row], dr[row]), np.flatnonzero(row & (fr != dr))[:5]
    # the fast bounds decide almost every random lookup (not the rows _dirs put on
    # an axis -- x = 0 or z = -0 is u on a texel edge -- nor the edge set)
    i = np.arange(300_000)
    plain = (i % 13 != 0) & (i % 17 != 0) & (i % 19 != 0) & (i % 23 != 0)
    assert col[i][plain].mean() > 0.99 and row[i][plain].mean() > 0.99, (col[i][plain].mean(), row[i][plain].mean())
