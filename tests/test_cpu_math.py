"""Parity trig (tinypathtracer_amd/csrc/common/ptrig.hpp) on the CPU.

* fsincos_2pi: the kernel's fp32 sin/cos of phi = 2*pi*u.  The header is
  compiled for the host with g++ (the same source the HIP kernel compiles) and
  must agree bit for bit with the oracle's C restatement (trig_mode 1), and
  stay within 1 ulp of the correctly rounded value over the curand input set.
* datan2 / dacos (env lookup): (float) of the double evaluation must equal
  (float) libm's double atan2/acos.
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
    for fn in ("h_sincos", "h_atan2", "h_acos"):
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
