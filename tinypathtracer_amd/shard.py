"""Pixel-band sharding across GPUs (one process per GPU) + framebuffer gather.

Rows are dealt in bands of `band_rows`.  The default deal interleaves them
(band b -> rank b % world) so miss-heavy and hit-heavy rows spread evenly; a
cost deal (cost_deal) balances the ranks by the bands' measured trace costs
from a previous frame (tpt_params.band_cost), for frames whose heavy rows the
interleave leaves on a few ranks.  The RNG subsequence is the global pixel
index (path_tracer.cu:39, :320), so any partition renders the same pixels
bit-identically to a single GPU.

A deal is a list, per rank, of ascending global band ids (tpt_params.band_list);
deal=None everywhere below means the interleaved one.

Two exchanges (RCCL over xGMI on the GPU box, gloo in the CPU tests):
  * gather_frame: one frame split across the ranks (strong scaling) -> one
    gather of each rank's compacted band rows into rank 0;
  * exchange_frames: a batch of N frames (one per rank, independent seeds, as
    the reference re-seeds every frame), each split across all N ranks so
    every GPU holds the same pixel mix as a whole frame (weak scaling) -> one
    all-to-all leaves frame f on rank f.
"""
from __future__ import annotations

import numpy as np


def n_bands(height: int, band_rows: int) -> int:
    return (height + band_rows - 1) // band_rows


def interleaved_deal(height: int, band_rows: int, world: int):
    """The default deal as explicit lists: band b -> rank b % world."""
    return [list(range(r, n_bands(height, band_rows), world)) for r in range(world)]


def band_row_ids(height: int, band_rows: int, world: int, rank: int, deal=None) -> np.ndarray:
    """Global row indices (row 0 = bottom) rendered by `rank`."""
    y = np.arange(height)
    if deal is None:
        return y[(y // band_rows) % world == rank]
    return y[np.isin(y // band_rows, np.asarray(deal[rank], dtype=np.int64))]


def max_band_height(height: int, band_rows: int, world: int, deal=None) -> int:
    return max(len(band_row_ids(height, band_rows, world, r, deal)) for r in range(world))


def cost_deal(costs, world: int, max_iter: int = 2000, order: str = "ascending", short_band=None, nset: int = 3):
    """Bands -> ranks by their measured costs (one float per global band, e.g.
    the summed wave life tpt_params.band_cost reports for the previous frame):
    longest-processing-time first -- heaviest band to the least-loaded rank --
    with every rank capped at ceil(bands / world) bands, so no rank holds more
    pixels than the interleaved deal's largest share (the lane-mode rules of
    tpt_render key on a launch's pixels); then pairwise swaps and moves that
    lower the larger of the two ranks' loads while the most loaded rank
    improves.  Deterministic (ties by band id, then rank id), so every rank
    computes the same deal from the same costs.  Returns per rank its band ids:
    ascending (order "ascending"), or heaviest first (order "heavy_first": the
    rank's launches dispatch its costliest bands first, so they do not end the
    frame); a short last band (short_band) stays last either way, as
    tpt_params.band_list requires."""
    c = [float(v) for v in costs]
    nb = len(c)
    if world < 1:
        raise ValueError("world >= 1")
    cap = (nb + world - 1) // world
    own = [[] for _ in range(world)]
    load = [0.0] * world
    for b in sorted(range(nb), key=lambda i: (-c[i], i)):
        r = min((r for r in range(world) if len(own[r]) < cap), key=lambda r: (load[r], r))
        own[r].append(b)
        load[r] += c[b]
    for _ in range(max_iter):
        m = max(range(world), key=lambda r: (load[r], -r))
        best = None   # (new max of the pair, band out, rank in, band back or -1)
        for i in own[m]:
            for r in range(world):
                if r == m:
                    continue
                if len(own[r]) < cap:   # move band i to rank r
                    pm = max(load[m] - c[i], load[r] + c[i])
                    if pm < load[m] and (best is None or pm < best[0]):
                        best = (pm, i, r, -1)
                for j in own[r]:        # swap band i with rank r's band j
                    d = c[i] - c[j]
                    if d <= 0.0:
                        continue
                    pm = max(load[m] - d, load[r] + d)
                    if pm < load[m] and (best is None or pm < best[0]):
                        best = (pm, i, r, j)
        if best is None:
            break
        _, i, r, j = best
        own[m].remove(i)
        own[r].append(i)
        load[m] -= c[i]
        load[r] += c[i]
        if j >= 0:
            own[r].remove(j)
            own[m].append(j)
            load[r] -= c[j]
            load[m] += c[j]
    if order == "ascending":
        return [sorted(o) for o in own]
    if order == "sets":
        return [set_balanced_order(o, c, nset, short_band) for o in own]
    if order != "heavy_first":
        raise ValueError("order: ascending, heavy_first or sets")
    return [sorted(o, key=lambda b: (b == short_band, -c[b], b)) for o in own]


def set_balanced_order(bands, costs, nset: int = 3, short_band=None):
    """One rank's bands ordered so that the launch pipeline's band sets carry
    equal costs.  tpt_render splits a listed share into nset sets on their own
    streams, set k taking list entries k, k + nset, ... (api.cpp); the sets run
    side by side and the last one to finish ends the frame, so a share whose
    bands do not divide evenly -- or whose few light bands fall into one set --
    ends on its heaviest set.  Set k gets ceil((n - k) / nset) slots; the bands
    fill them longest-processing-time first (heaviest band to the least-loaded
    set with a free slot); a short last band is placed in the set that holds
    the list's last slot.  Each set keeps its bands in ascending order, and the
    list interleaves the sets, so list[k::nset] is set k.  Deterministic."""
    bands = [int(b) for b in bands]
    n = len(bands)
    if nset <= 1 or n <= 1:
        return sorted(bands, key=lambda b: (b == short_band, b))
    nset = min(nset, n)
    size = [(n - k + nset - 1) // nset for k in range(nset)]
    groups = [[] for _ in range(nset)]
    load = [0.0] * nset
    rest = bands
    if short_band is not None and short_band in bands:
        k = (n - 1) % nset
        groups[k].append(short_band)
        load[k] += float(costs[short_band])
        rest = [b for b in bands if b != short_band]
    for b in sorted(rest, key=lambda i: (-float(costs[i]), i)):
        k = min((k for k in range(nset) if len(groups[k]) < size[k]), key=lambda k: (load[k], k))
        groups[k].append(b)
        load[k] += float(costs[b])
    for g in groups:
        g.sort(key=lambda b: (b == short_band, b))
    out = []
    for i in range(max(size)):
        for k in range(nset):
            if i < len(groups[k]):
                out.append(groups[k][i])
    return out


def deal_loads(costs, deal):
    """Summed cost per rank of a deal (its predicted balance)."""
    return [float(sum(costs[b] for b in d)) for d in deal]


def gather_frame(radiance, height: int, band_rows: int, world: int, rank: int, dist=None, group=None, deal=None):
    """Gather every rank's band rows of `radiance` [H, W, C] (torch tensor) into
    rank 0.  Returns the assembled frame on rank 0, None elsewhere.

    Each rank packs its rows into a [maxH, W, C] slab (padding rows zero), one
    gather moves the slabs, rank 0 scatters rows back with index_copy."""
    import torch

    if dist is None:
        import torch.distributed as dist
    rows = band_row_ids(height, band_rows, world, rank, deal)
    mh = max_band_height(height, band_rows, world, deal)
    w, c = radiance.shape[1], radiance.shape[2]
    slab = radiance.new_zeros((mh, w, c))
    idx = torch.as_tensor(rows, device=radiance.device, dtype=torch.long)
    slab[: len(rows)] = radiance.index_select(0, idx)
    if world == 1:
        return radiance
    if rank == 0:
        slabs = [radiance.new_empty((mh, w, c)) for _ in range(world)]
        dist.gather(slab, gather_list=slabs, dst=0, group=group)
        out = radiance.new_zeros(radiance.shape)
        for r in range(world):
            rr = band_row_ids(height, band_rows, world, r, deal)
            ri = torch.as_tensor(rr, device=radiance.device, dtype=torch.long)
            out.index_copy_(0, ri, slabs[r][: len(rr)])
        return out
    dist.gather(slab, gather_list=None, dst=0, group=group)
    return None


def exchange_frames(radiances, height: int, band_rows: int, world: int, rank: int, dist=None, group=None,
                    deal=None):
    """Weak-scaling exchange for a batch of `world` frames: rank r rendered its
    band rows of every frame f (radiances[f], [H, W, C] tensors); one
    all-to-all (RCCL over xGMI: every rank sends to every peer at once, one
    xGMI link each) leaves frame f whole on rank f.  Returns this rank's frame.

    Each rank packs its rows of each frame into a [world, maxH, W, C] stack
    (padding rows zero); slot f goes to rank f; the received slot r holds rank
    r's rows of this rank's frame."""
    import torch

    if dist is None:
        import torch.distributed as dist
    if len(radiances) != world:
        raise ValueError("exchange_frames: one frame per rank")
    if world == 1:
        return radiances[0]
    rows = band_row_ids(height, band_rows, world, rank, deal)
    mh = max_band_height(height, band_rows, world, deal)
    ref = radiances[0]
    w, c = ref.shape[1], ref.shape[2]
    idx = torch.as_tensor(rows, device=ref.device, dtype=torch.long)
    send = ref.new_zeros((world, mh, w, c))
    for f in range(world):
        send[f, : len(rows)] = radiances[f].index_select(0, idx)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=group)
    out = ref.new_zeros(ref.shape)
    for r in range(world):
        rr = band_row_ids(height, band_rows, world, r, deal)
        ri = torch.as_tensor(rr, device=ref.device, dtype=torch.long)
        out.index_copy_(0, ri, recv[r, : len(rr)])
    return out
