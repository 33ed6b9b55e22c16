"""Pixel-band sharding across GPUs (one process per GPU) + framebuffer gather.

Rows are dealt in interleaved bands of `band_rows` (band b -> rank b % world)
so miss-heavy and hit-heavy rows spread evenly.  The RNG subsequence is the
global pixel index (path_tracer.cu:39, :320), so any partition renders the
same pixels bit-identically to a single GPU.

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


def band_row_ids(height: int, band_rows: int, world: int, rank: int) -> np.ndarray:
    """Global row indices (row 0 = bottom) rendered by `rank`."""
    y = np.arange(height)
    return y[(y // band_rows) % world == rank]


def max_band_height(height: int, band_rows: int, world: int) -> int:
    return max(len(band_row_ids(height, band_rows, world, r)) for r in range(world))


def gather_frame(radiance, height: int, band_rows: int, world: int, rank: int, dist=None, group=None):
    """Gather every rank's band rows of `radiance` [H, W, C] (torch tensor) into
    rank 0.  Returns the assembled frame on rank 0, None elsewhere.

    Each rank packs its rows into a [maxH, W, C] slab (padding rows zero), one
    gather moves the slabs, rank 0 scatters rows back with index_copy."""
    import torch

    if dist is None:
        import torch.distributed as dist
    rows = band_row_ids(height, band_rows, world, rank)
    mh = max_band_height(height, band_rows, world)
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
            rr = band_row_ids(height, band_rows, world, r)
            ri = torch.as_tensor(rr, device=radiance.device, dtype=torch.long)
            out.index_copy_(0, ri, slabs[r][: len(rr)])
        return out
    dist.gather(slab, gather_list=None, dst=0, group=group)
    return None


def exchange_frames(radiances, height: int, band_rows: int, world: int, rank: int, dist=None, group=None):
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
    rows = band_row_ids(height, band_rows, world, rank)
    mh = max_band_height(height, band_rows, world)
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
        rr = band_row_ids(height, band_rows, world, r)
        ri = torch.as_tensor(rr, device=ref.device, dtype=torch.long)
        out.index_copy_(0, ri, recv[r, : len(rr)])
    return out
