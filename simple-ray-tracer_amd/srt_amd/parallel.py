"""Multi-GPU frame tiling: row bands dealt round-robin to ranks + one gather to the root.

Pixels are independent and every random number is a pure function of (global pixel, frame,
hit position), so rank r renders bands b with b % nranks == r (bands of `band_rows` rows,
8x8-tile aligned) with global coordinates and the frame is bit-identical to a 1-GPU render.
Per frame the only exchange is one gather of each rank's packed sRGB8 rows (every rank encodes its
own rows: accumFrames is one uniform) to the root (torch.distributed: RCCL over xGMI with the
"nccl" backend, gloo on CPU), which de-interleaves them (srt_assemble_output_bands on the GPU).
The radiance rows (RGBA32F, 4x the bytes) stay on their rank and are gathered only when the full
accumulation image is wanted (srt_assemble_bands).
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


def gather_bands(local, dst: int = 0, collective: bool = False, out=None):
    """Gather every rank's equal-size band buffer to `dst` (one collective).  Returns the
    [nranks, ...] tensor on dst (`out` when given: a preallocated receive buffer whose rank slices
    the collective writes in place, so the root makes no stacking copy), None elsewhere.  One rank
    skips the collective unless `collective` (the one-GPU test of the RCCL path)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    rank = dist.get_rank()
    if world == 1 and not collective:
        if out is None:
            return local.unsqueeze(0)
        out[0].copy_(local)
        return out
    # gloo gathers host tensors: a device buffer is staged through the host and the result moved
    # back (multi-rank tests on one GPU); RCCL ("nccl") gathers device memory directly over xGMI
    staged = dist.get_backend() == "gloo" and local.is_cuda
    src = local.cpu() if staged else local
    recv = None
    if rank == dst:
        if out is not None and not staged:
            recv = out
        else:
            recv = torch.empty((world,) + tuple(src.shape), dtype=src.dtype, device=src.device)
    dist.gather(src, list(recv.unbind(0)) if recv is not None else None, dst=dst)
    if rank != dst:
        return None
    if staged:
        if out is not None:
            out.copy_(recv)
            return out
        return recv.to(local.device)
    return recv
