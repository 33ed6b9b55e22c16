"""CPU tests of the SAH 4-wide traversal tree (host/wide_bvh.cpp, exported as
tpt_wide_tree_build) that tpt_scene_build uploads for the ordered traversal.

The tree is exact only if (1) its leaves are the LBVH's leaves -- every sorted
position exactly once, carrying the reference's own leaf box bit for bit
(bvh.cu:128-148) -- and (2) every inner box contains its subtree, so a leaf
whose box passes the slab test is reached (path_tracer.cu:61-107 reaches a
leaf iff its box and its ancestors' boxes pass, and for finite rays the
ancestors pass whenever the leaf does).  Both are checked here on the shipped
scenes and the synthesized C5 scene, plus a brute-force reachability check on
random rays."""
import ctypes as C

import numpy as np
import pytest

import tinypathtracer_amd as T
from oracle import oracle as O
from tests.conftest import scene_path


def _leaves(name):
    ps = O.load_scene(scene_path(name))
    nodes, _, _, _ = O.build_bvh(ps)
    n = len(ps.indices) // 3
    lf = nodes[n - 1:]
    box = np.concatenate([lf["bmin"], lf["bmax"]], axis=1).astype(np.float32)   # by sorted position
    s = ps.src
    mats = np.asarray(s.materials, np.float32).reshape(-1, 15) if len(s.materials) else np.zeros((0, 15), np.float32)
    emit = np.zeros(n, np.uint32)
    for pos, fid in enumerate(lf["a"]):
        obj = max(i for i, (b, _) in enumerate(s.lut) if fid >= b) if any(fid >= b for b, _ in s.lut) else -1
        m = s.lut[obj][1] if obj >= 0 else -1
        e = mats[m][3] if 0 <= m < len(mats) else 0.0
        emit[pos] = 1 if e != 0.0 else 0
    return n, box, emit


def _build(n, box, emit, threads=-1):
    lib = T.lib()
    lv = C.c_int32(0)
    cnt = lib.tpt_wide_tree_build(n, box.ctypes.data, emit.ctypes.data, None, 0, C.byref(lv), threads)
    assert cnt > 0
    out = np.zeros((cnt, 32), np.float32)
    assert lib.tpt_wide_tree_build(n, box.ctypes.data, emit.ctypes.data, out.ctypes.data, cnt, C.byref(lv),
                                   threads) == cnt
    return out, lv.value


def _check(n, box, emit, out, need):
    n4 = len(out)
    nint = n - 1
    assert n4 <= nint
    links = out[:, 24:28].view(np.int32)
    seen_leaf = np.zeros(n, np.int32)
    seen_node = np.zeros(n4, np.int32)
    seen_node[0] = 1   # root
    above = np.full(n4, -1)   # stack entries a visit can find: deferred siblings of the node and its ancestors
    above[0] = 0
    nk = (links >= 0).sum(1)
    # breadth-first numbering: children have larger ids than their parent
    for i in range(n4):
        kids = 0
        for k in range(4):
            L = int(links[i, k])
            if L < 0:
                assert not out[i, 6 * k:6 * k + 6].any()
                continue
            kids += 1
            cid, ef = L & 0x3fffffff, (L >> 30) & 1
            cb = out[i, 6 * k:6 * k + 6]
            if cid >= nint:
                pos = cid - nint
                seen_leaf[pos] += 1
                assert np.array_equal(cb.view(np.uint32), box[pos].view(np.uint32))   # the reference's leaf box
                assert ef == emit[pos]
            else:
                assert cid > i
                seen_node[cid] += 1
                above[cid] = above[i] + nk[i] - 1
                sub = out[cid].reshape(-1)[:24].reshape(4, 6)
                sl = links[cid]
                valid = sl >= 0
                assert (cb[:3] <= sub[valid, :3]).all() and (cb[3:] >= sub[valid, 3:]).all()
                assert ef == int(((sl[valid] >> 30) & 1).max())
        assert kids >= 2
    assert (seen_leaf == 1).all()
    assert (seen_node == 1).all()
    assert (above >= 0).all()
    assert int((above + nk - 1).max()) == need


@pytest.mark.parametrize("name", ["box", "ball", "tir", "box2", "light", "square", "c5"])
def test_wide_tree_structure(name):
    n, box, emit = _leaves(name)
    out, need = _build(n, box, emit)
    _check(n, box, emit, out, need)
    assert need <= 150   # the kernel's stack capacity
    # nodes are mostly full (the collapse opens internal children until 4)
    links = out[:, 24:28].view(np.int32)
    if n >= 64:
        assert (links >= 0).sum(1).mean() > 3.5


def _slab_pass(o, inv, b, hd=np.float32(1e-4)):
    """min/max slab test of trace.hip's inner_visit4 (finite ray): hit and exit >= Delta/2."""
    a = (b[..., :3] - o) * inv
    c = (b[..., 3:] - o) * inv
    t0 = np.minimum(a, c).max(-1)
    t1 = np.maximum(a, c).min(-1)
    return np.maximum(t0, hd) <= np.minimum(t1, np.float32(3.4028235e38))


def test_wide_tree_reaches_every_passing_leaf():
    n, box, emit = _leaves("box")
    out, _ = _build(n, box, emit)
    links = out[:, 24:28].view(np.int32)
    nint = n - 1
    rng = np.random.default_rng(5)
    lo, hi = box[:, :3].min(0), box[:, 3:].max(0)
    for _ in range(64):
        o = (lo + (hi - lo) * rng.random(3)).astype(np.float32)
        d = rng.normal(size=3).astype(np.float32)
        d /= np.float32(np.linalg.norm(d))
        inv = (np.float32(1.0) / d).astype(np.float32)
        want = set(np.nonzero(_slab_pass(o, inv, box))[0].tolist())
        got, stack = set(), [0]
        while stack:
            i = stack.pop()
            bx = out[i, :24].reshape(4, 6)
            ok = _slab_pass(o, inv, bx)
            for k in range(4):
                L = int(links[i, k])
                if L < 0 or not ok[k]:
                    continue
                cid = L & 0x3fffffff
                if cid >= nint:
                    got.add(cid - nint)
                else:
                    stack.append(cid)
        assert got == want


def _random_leaves(n, seed):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-50.0, 50.0, (n, 3)).astype(np.float32)
    e = rng.uniform(0.01, 2.0, (n, 3)).astype(np.float32)
    box = np.concatenate([c - e, c + e], axis=1).astype(np.float32)
    emit = (rng.random(n) < 0.01).astype(np.uint32)
    return box, emit


@pytest.mark.parametrize("case", ["c5", "random"])
def test_threaded_build_equals_serial_build(case):
    """The threaded SAH build (subtrees of >= 4096 leaves on their own threads,
    host/wide_bvh.cpp) writes the same node array as the serial build, byte for
    byte, for every thread count -- pre-order ids are fixed before a subtree is
    built, so only the schedule differs."""
    if case == "c5":
        n, box, emit = _leaves("c5")
    else:
        n = 40000
        box, emit = _random_leaves(n, 11)
    serial, need = _build(n, box, emit, threads=0)
    assert n > 8192   # large enough that the threaded path spawns
    for threads in (1, 2, 3, 8, 32, -1):
        got, need2 = _build(n, box, emit, threads=threads)
        assert need2 == need
        assert got.tobytes() == serial.tobytes(), threads
