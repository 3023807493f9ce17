"""Multi-GPU frame tiling: row bands dealt round-robin to ranks + one gather to the root.

Pixels are independent and every random number is a pure function of (global pixel, frame,
hit position), so rank r renders bands b with b % nranks == r (bands of `band_rows` rows,
8x8-tile aligned) with global coordinates and the frame is bit-identical to a 1-GPU render.
The only exchange is one gather of each rank's packed radiance rows (RGBA32F) to the root
(torch.distributed: RCCL over xGMI with the "nccl" backend, gloo on CPU), after which the root
de-interleaves the bands and encodes sRGB8 (srt_assemble_bands on the GPU).
"""
from __future__ import annotations

import numpy as np


def num_bands(height: int, band_rows: int) -> int:
    return (height + band_rows - 1) // band_rows


def rows_pad(height: int, band_rows: int, nranks: int) -> int:
    """Rows of the (padded, equal-size) per-rank buffer the gather moves."""
    return ((num_bands(height, band_rows) + nranks - 1) // nranks) * band_rows


def local_global_rows(height: int, band_rows: int, nranks: int, rank: int) -> np.ndarray:
    """Global row of each packed local row of `rank` (the kernel's ly -> gy mapping)."""
    rows = []
    for b in range(rank, num_bands(height, band_rows), nranks):
        rows.extend(range(b * band_rows, min((b + 1) * band_rows, height)))
    return np.asarray(rows, np.int64)


def assemble_host(gathered: np.ndarray, height: int, band_rows: int) -> np.ndarray:
    """Host restatement of srt_assemble_bands' de-interleave: gathered[rank, local_row] -> frame."""
    nranks = gathered.shape[0]
    out = np.zeros((height,) + gathered.shape[2:], gathered.dtype)
    for r in range(nranks):
        g = local_global_rows(height, band_rows, nranks, r)
        out[g] = gathered[r, :len(g)]
    return out


def gather_bands(local, dst: int = 0, collective: bool = False):
    """Gather every rank's equal-size band buffer to `dst` (one collective).  Returns the stacked
    [nranks, ...] tensor on dst, None elsewhere.  One rank skips the collective unless `collective`
    (the one-GPU test of the RCCL path)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    if world == 1 and not collective:
        return local.unsqueeze(0)
    # gloo gathers host tensors: a device buffer is staged through the host and the stacked result
    # moved back (multi-rank tests on one GPU); RCCL ("nccl") gathers device memory directly over xGMI
    staged = dist.get_backend() == "gloo" and local.is_cuda
    src = local.cpu() if staged else local
    parts = [torch.empty_like(src) for _ in range(world)] if rank == dst else None
    dist.gather(src, parts, dst=dst)
    if rank != dst:
        return None
    stacked = torch.stack(parts)
    return stacked.to(local.device) if staged else stacked
