"""Multi-rank sharding on CPU (gloo, world size 2 and 3): each rank renders its
interleaved row bands with the CPU oracle (standing in for the GPU render) and
tinypathtracer_amd.shard.gather_frame assembles the frame on rank 0 -- it must
be bit-identical to the single-process frame (the RNG subsequence is the
global pixel index, path_tracer.cu:39,320)."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP, BAND = 40, 37, 4, 8


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out_path):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from tinypathtracer_amd import shard
    ps = O.load_scene(os.path.join(ROOT, "tests", "golden", "scenes", "box.gltf"))
    rad, _, _ = O.render(ps, W, H, SPP, 8, 42, trig_mode=1, band_rows=BAND, band_count=world, band_index=rank,
                         threads=1)
    frame = shard.gather_frame(torch.from_numpy(rad), H, BAND, world, rank)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_band_gather_bit_identical(tmp_path, world):
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    ps = O.load_scene(os.path.join(ROOT, "tests", "golden", "scenes", "box.gltf"))
    full, _, _ = O.render(ps, W, H, SPP, 8, 42, trig_mode=1)
    got = np.load(out)
    assert np.array_equal(got.view(np.uint32), full.view(np.uint32))


def test_band_rows_partition():
    from tinypathtracer_amd import shard
    for world in (1, 2, 3, 4, 8):
        rows = np.concatenate([shard.band_row_ids(1080, 16, world, r) for r in range(world)])
        assert sorted(rows.tolist()) == list(range(1080))
        hs = [len(shard.band_row_ids(1080, 16, world, r)) for r in range(world)]
        assert max(hs) - min(hs) <= 16


def _worker_frames(rank, world, port, out_dir):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from tinypathtracer_amd import shard
    ps = O.load_scene(os.path.join(ROOT, "tests", "golden", "scenes", "box.gltf"))
    # weak scaling: this rank's bands of every frame of the batch (frame f: seed 42 + f)
    rads = [torch.from_numpy(O.render(ps, W, H, SPP, 8, 42 + f, trig_mode=1, band_rows=BAND, band_count=world,
                                      band_index=rank, threads=1)[0]) for f in range(world)]
    frame = shard.exchange_frames(rads, H, BAND, world, rank)
    np.save(os.path.join(out_dir, f"frame{rank}.npy"), frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_frame_batch_all_to_all(tmp_path, world):
    """Frame batch across ranks (bench.py weak scaling): after the all-to-all,
    rank f holds frame f (seed 42 + f) bit-identical to a one-process render."""
    mp.start_processes(_worker_frames, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    ps = O.load_scene(os.path.join(ROOT, "tests", "golden", "scenes", "box.gltf"))
    for f in range(world):
        full, _, _ = O.render(ps, W, H, SPP, 8, 42 + f, trig_mode=1)
        got = np.load(str(tmp_path / f"frame{f}.npy"))
        assert np.array_equal(got.view(np.uint32), full.view(np.uint32)), f


def test_cost_deal_partitions_and_balances():
    """shard.cost_deal: every band dealt exactly once, ascending per rank, at most
    ceil(bands / world) bands per rank (no rank holds more pixels than the
    interleaved deal's largest share), deterministic, and its most loaded rank
    no heavier than the interleaved deal's (strictly lighter on skewed costs)."""
    from tinypathtracer_amd import shard
    rng = np.random.default_rng(7)
    for nb, world in ((68, 8), (135, 8), (68, 4), (9, 2), (5, 8), (1, 3)):
        costs = (rng.random(nb) ** 4 * 100.0).astype(np.float32)
        costs[nb // 2: nb // 2 + 3] *= 20.0   # a few heavy rows in the middle, as on box and C5
        d = shard.cost_deal(costs, world)
        assert len(d) == world
        assert sorted(b for r in d for b in r) == list(range(nb))
        assert all(r == sorted(r) for r in d)
        assert max(len(r) for r in d) <= -(-nb // world)
        assert d == shard.cost_deal(costs, world)
        inter = [list(range(r, nb, world)) for r in range(world)]
        assert max(shard.deal_loads(costs, d)) <= max(shard.deal_loads(costs, inter)) + 1e-3
        if nb >= 4 * world:
            assert max(shard.deal_loads(costs, d)) < max(shard.deal_loads(costs, inter))
    # the deal's rows partition the frame, and band_row_ids follows the deal
    d = shard.cost_deal(rng.random(68), 8)
    rows = np.concatenate([shard.band_row_ids(1080, 16, 8, r, d) for r in range(8)])
    assert sorted(rows.tolist()) == list(range(1080))
    assert shard.interleaved_deal(1080, 16, 8)[3] == list(range(3, 68, 8))


def test_set_balanced_order():
    """shard.set_balanced_order: a permutation of the rank's bands whose
    list[k::nset] (tpt_render's band set k) are ascending, sized
    ceil((n - k) / nset), with a short last band last; the sets' cost spread is
    at most one band's cost, and no larger than the plain ascending order's."""
    from tinypathtracer_amd import shard
    rng = np.random.default_rng(11)
    costs = rng.random(135) * 100.0
    costs[[0, 134]] = 0.5   # nearly empty top and bottom bands, as at C5
    for bands, nset, short in ((list(range(7, 135, 8)), 3, None), (list(range(0, 135, 8)), 3, None),
                               (list(range(135)), 3, None), (list(range(3, 68, 4)), 2, 67), (list(range(9)), 4, 8),
                               ([5], 3, None), ([], 3, None)):
        o = shard.set_balanced_order(bands, costs, nset, short)
        assert sorted(o) == sorted(bands)
        if short is not None:
            assert o[-1] == short
        k_sets = min(nset, max(len(o), 1))
        if len(o) <= 1:
            continue
        sets = [o[k::k_sets] for k in range(k_sets)]
        assert all(s_ == sorted(s_, key=lambda b: (b == short, b)) for s_ in sets)
        assert [len(s_) for s_ in sets] == [(len(o) - k + k_sets - 1) // k_sets for k in range(k_sets)]
        loads = [sum(costs[b] for b in s_) for s_ in sets]
        plain = sorted(bands, key=lambda b: (b == short, b))
        ploads = [sum(costs[b] for b in plain[k::k_sets]) for k in range(k_sets)]
        assert max(loads) - min(loads) <= max(costs[b] for b in bands) + 1e-9
        assert max(loads) <= max(ploads) + 1e-9
    # through cost_deal
    d = shard.cost_deal(costs, 8, order="sets", nset=3)
    assert sorted(b for r in d for b in r) == list(range(135))


def _worker_deal(rank, world, port, out_path, deal):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    from tinypathtracer_amd import shard
    ps = O.load_scene(os.path.join(ROOT, "tests", "golden", "scenes", "box.gltf"))
    nb = shard.n_bands(H, BAND)
    rad = np.zeros((H, W, 3), np.float32)
    for b in deal[rank]:   # this rank's bands of the explicit deal, one oracle band render each
        rb, _, _ = O.render(ps, W, H, SPP, 8, 42, trig_mode=1, band_rows=BAND, band_count=nb, band_index=b,
                            threads=1)
        rows = shard.band_row_ids(H, BAND, nb, b)
        rad[rows] = rb[rows]
    frame = shard.gather_frame(torch.from_numpy(rad), H, BAND, world, rank, deal=deal)
    if rank == 0:
        np.save(out_path, frame.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_cost_deal_gather_bit_identical(tmp_path, world):
    """A non-interleaved deal (shard.cost_deal of skewed costs): each rank
    renders its bands, gather_frame(deal=...) assembles rank 0's frame, bit for
    bit the one-process frame."""
    from tinypathtracer_amd import shard
    nb = shard.n_bands(H, BAND)
    costs = np.array([1.0, 9.0, 8.0, 1.0, 0.5][:nb] + [0.1] * max(0, nb - 5), np.float32)
    deal = shard.cost_deal(costs, world)
    assert deal != shard.interleaved_deal(H, BAND, world)
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker_deal, args=(world, _free_port(), out, deal), nprocs=world, join=True,
                       start_method="spawn")
    from oracle import oracle as O
    ps = O.load_scene(os.path.join(ROOT, "tests", "golden", "scenes", "box.gltf"))
    full, _, _ = O.render(ps, W, H, SPP, 8, 42, trig_mode=1)
    assert np.array_equal(np.load(out).view(np.uint32), full.view(np.uint32))


def test_bench_refuses_gpus_that_disagree_with_world_size():
    """bench.py under an external launcher: a --gpus that differs from WORLD_SIZE
    exits non-zero before any GPU or torch work (so a driver that asks for N GPUs
    never silently times one); runs on the CPU."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr, (r.returncode, r.stderr[-500:])
