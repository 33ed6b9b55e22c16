"""Pixel-band sharding across GPUs (one process per GPU) + framebuffer gather.

Rows are dealt in interleaved bands of `band_rows` (band b -> rank b % world)
so miss-heavy and hit-heavy rows spread evenly.  The RNG subsequence is the
global pixel index (path_tracer.cu:39, :320), so any partition renders the
same pixels bit-identically to a single GPU.  The only exchange is one gather
of each rank's compacted band rows into rank 0 (RCCL over xGMI on the GPU box,
gloo in the CPU tests).
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
