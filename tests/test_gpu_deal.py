"""Explicit band deals on the GPU (tpt_params.band_list / band_cost; DESIGN.md
section 6 "Cost-balanced deal").

A deal hands each rank any set of whole bands; the RNG subsequence is the
global pixel index (path_tracer.cu:39,320), so every deal must assemble the
one-GPU frame bit for bit -- with one launch, with the launch pipeline's band
sets (each set takes every nset-th entry of the rank's list), with four lanes
per pixel and in pair mode, for frame batches and progressive accumulation.
band_cost reports a positive cost for exactly the bands a call rendered.
"""
import numpy as np
import pytest

import tinypathtracer_amd as T
from tests.conftest import scene_path
from tinypathtracer_amd import shard

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _skewed_deal(nb, world, seed=3, order="ascending", short_band=None):
    rng = np.random.default_rng(seed)
    costs = rng.random(nb).astype(np.float32) ** 3
    d = shard.cost_deal(costs, world, order=order, short_band=short_band)
    assert d != shard.interleaved_deal(nb * 16, 16, world)
    return d


@pytest.mark.parametrize("scene,W,H,spp,kw", [
    ("box", 256, 144, 16, {}),
    ("box", 256, 144, 16, {"lanes_per_pixel": 4}),
    ("box", 256, 150, 16, {"pipe_sets": 3, "pipe_chunks": 2}),      # partial last band, three band sets
    ("ball", 256, 144, 16, {}),                                     # pair mode (delta light)
    ("tir", 200, 120, 32, {"lanes_per_pixel": 1, "pipe_sets": 2, "pipe_chunks": 4}),
    ("box", 192, 112, 8, {"flags": 0x20}),                          # the wavefront variant (no band costs)
])
def test_explicit_deal_bit_identical(scene, W, H, spp, kw):
    s = T.Scene(scene_path(scene))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        if scene == "ball":
            pt.envLight = T.EnvLight(T.procedural_sky(256, 128), 0)
        full = np.zeros((H, W, 3), np.float32)
        st = pt.doTrace(d, s.m_camera, None, spp, seed=42, radiance=full)
        nb = shard.n_bands(H, 16)
        for world in (2, 3):
            # world 3: each rank's bands heaviest first (dispatch order = list order), a
            # short last band last
            deal = _skewed_deal(nb, world, order="ascending" if world == 2 else "heavy_first",
                                short_band=nb - 1 if H % 16 else None)
            acc = np.zeros((H, W, 3), np.float32)
            rays = 0
            for r in range(world):
                cost = np.zeros(nb, np.float32)
                st_r = pt.doTrace(d, s.m_camera, None, spp, seed=42, radiance=acc, band=(16, world, r),
                                  band_list=deal[r], band_cost=cost, **kw)
                rays += st_r["traversals"]
                mine = np.zeros(nb, bool)
                mine[deal[r]] = True
                if kw.get("flags", 0) & T._lib.FLAG_WAVEFRONT:
                    assert (cost == 0).all()   # (megakernel only, tpt.h)
                else:
                    assert (cost[mine] > 0).all() and (cost[~mine] == 0).all(), (r, cost)
                assert st_r["pixels"] == W * len(shard.band_row_ids(H, 16, world, r, deal))
            assert int((_bits(acc) != _bits(full)).any(-1).sum()) == 0, (scene, world, kw)
            assert rays == st["traversals"]
    finally:
        d.close()


def test_explicit_deal_frames_and_accumulate():
    """A frame batch and a progressive continuation under an explicit deal."""
    W, H, spp = 192, 112, 8
    s = T.Scene(scene_path("box"))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        seeds = [42, 43]
        fulls = [np.zeros((H, W, 3), np.float32) for _ in seeds]
        pt.doTraceFrames(d, s.m_camera, seeds, None, spp, radiances=fulls)
        deal = _skewed_deal(shard.n_bands(H, 16), 2)
        accs = [np.zeros((H, W, 3), np.float32) for _ in seeds]
        for r in range(2):
            pt.doTraceFrames(d, s.m_camera, seeds, None, spp, radiances=accs, band=(16, 2, r), band_list=deal[r])
        for f in range(2):
            assert np.array_equal(_bits(accs[f]), _bits(fulls[f])), f
        # progressive: 2 x 4 spp under the deal == 8 spp in one call
        acc = np.zeros((H, W, 3), np.float32)
        pt.doTrace(d, s.m_camera, None, 4, seed=42, radiance=acc, band=(16, 2, 0), band_list=deal[0])
        pt.doTrace(d, s.m_camera, None, 4, seed=42, radiance=acc, band=(16, 2, 0), band_list=deal[0],
                   accumulate=True)
        rows = shard.band_row_ids(H, 16, 2, 0, deal)
        assert np.array_equal(_bits(acc[rows]), _bits(fulls[0][rows]))
    finally:
        d.close()


def test_band_list_refusals():
    W, H = 64, 40
    s = T.Scene(scene_path("box"))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        for bad in ([0, 0], [3], [-1], [2, 0]):   # duplicate, out of range, the short band not last
            with pytest.raises(T.TPTError):
                pt.doTrace(d, s.m_camera, None, 2, seed=1, band_list=bad)
        with pytest.raises(ValueError):
            pt.doTrace(d, s.m_camera, None, 2, seed=1, band_cost=np.zeros(2, np.float32))
        st = pt.doTrace(d, s.m_camera, None, 2, seed=1, band_list=[1, 0, 2])   # any order, short band last
        assert st["pixels"] == W * H
        # an empty list renders nothing
        st = pt.doTrace(d, s.m_camera, None, 2, seed=1, band_list=[])
        assert st["pixels"] == 0 and st["traversals"] == 0
    finally:
        d.close()


def test_full_size_c2_cost_deal_8_ways():
    """The strong-scaled C2 split (1920x1080x1024 spp, 8 ranks) with the cost deal
    bench.py uses: the costs of a probe frame in interleaved bands, then
    shard.cost_deal; the assembled frame equals the one-GPU frame bit for bit,
    the rays are the same, and the deal's predicted balance beats the
    interleave's."""
    W, H, spp, depth, N = 1920, 1080, 1024, 8, 8
    s = T.Scene(scene_path("box"))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        full = np.zeros((H, W, 3), np.float32)
        st = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=full)
        nb = shard.n_bands(H, 16)
        costs = np.zeros(nb, np.float32)
        for r in range(N):
            pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, band=(16, N, r), band_cost=costs)
        assert (costs > 0).all()
        deal = shard.cost_deal(costs, N)
        il = shard.deal_loads(costs, shard.interleaved_deal(H, 16, N))
        cl = shard.deal_loads(costs, deal)
        assert max(cl) <= max(il)
        acc = np.zeros((H, W, 3), np.float32)
        rays = 0
        for r in range(N):
            st_r = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=acc, band=(16, N, r),
                              band_list=deal[r])
            rays += st_r["traversals"]
            assert st_r["lanes_per_pixel"] == 4 and st_r["drained"] == 1   # 259 K pixels: four lanes
        assert int((_bits(acc) != _bits(full)).any(-1).sum()) == 0
        assert rays == st["traversals"]
        assert st["resident_lanes"] > 0
        # N = 2 (1 M pixels per rank: one lane per pixel, the full-occupancy variants, three
        # band sets), each rank's bands heaviest first
        deal2 = shard.cost_deal(costs, 2, order="heavy_first", short_band=nb - 1)
        acc2 = np.zeros((H, W, 3), np.float32)
        for r in range(2):
            st_r = pt.doTrace(d, s.m_camera, None, spp, seed=42, max_depth=depth, radiance=acc2, band=(16, 2, r),
                              band_list=deal2[r])
            assert st_r["lanes_per_pixel"] == 1 and st_r["drained"] == 0
        assert int((_bits(acc2) != _bits(full)).any(-1).sum()) == 0
    finally:
        d.close()


@pytest.mark.parametrize("W,H,kw", [
    (256, 96, {"pipe_sets": 2, "pipe_chunks": 4}),                       # XCD runs of 2 tiles, 4 rotations per set
    (640, 160, {"pipe_sets": 3, "pipe_chunks": 8, "band": (16, 2, 1), "lanes_per_pixel": 1}),   # runs of 5, one lane,
                                                                     # a strong-scaled share
])
def test_xcd_runs_rotated_per_chunk_bit_identical(W, H, kw):
    """A scene larger than an XCD's L2 (c5, 131 K triangles) deals tiles to XCDs in
    runs that rotate by one per chunk of a set's samples (api.cpp xcd_rot): the
    chunked, pipelined render equals one launch bit for bit."""
    s = T.Scene(scene_path("c5"))
    d = s.copySceneToDevice(0).build()
    try:
        pt = T.PathTracer("", W, H, 0)
        spp = 16
        band = kw.pop("band", (16, 1, 0))
        one = np.zeros((H, W, 3), np.float32)
        st1 = pt.doTrace(d, s.m_camera, None, spp, seed=7, radiance=one, band=band, pipe_sets=1,
                         spp_per_launch=spp, lanes_per_pixel=kw.get("lanes_per_pixel", 0))
        piped = np.zeros((H, W, 3), np.float32)
        st2 = pt.doTrace(d, s.m_camera, None, spp, seed=7, radiance=piped, band=band, **kw)
        assert st2["trace_launches"] > kw["pipe_sets"], st2   # several chunks per set
        assert st1["traversals"] == st2["traversals"]
        assert np.array_equal(_bits(piped), _bits(one))
    finally:
        d.close()
