"""Image-band sharding across ranks and the strip gather.

Rows are cut into bands of ``band_rows``; band b belongs to rank b % world (round-robin, so
the frog in the middle of the frame is spread over every GPU).  Each rank renders its bands
contiguously into a "strip" (the layout rt_render_device writes when band_count > 1); rank 0
gathers the strips (one collective: torch.distributed.gather, RCCL over xGMI on GPUs, gloo on
CPU) and un-permutes them into the frame.  Pixels are independent, so the assembled frame
is bit-identical to a single-GPU render.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np


def rows_of(height: int, band_rows: int, rank: int, world: int) -> List[int]:
    """Image rows owned by `rank`, in strip order (== rt_shard_rows row mapping)."""
    if world <= 1:
        return list(range(height))
    return [y for y in range(height) if (y // band_rows) % world == rank]


def bands_of(height: int, band_rows: int, rank: int, world: int):
    """(y0, y1) row ranges owned by `rank`, in strip order."""
    if world <= 1:
        return [(0, height)]
    nb = (height + band_rows - 1) // band_rows
    return [(b * band_rows, min(height, (b + 1) * band_rows)) for b in range(rank, nb, world)]


def max_strip_rows(height: int, band_rows: int, world: int) -> int:
    return max(len(rows_of(height, band_rows, r, world)) for r in range(world))


def gather_frame(strip, height: int, band_rows: int, world: int, rank: int, gather_list=None):
    """Gather every rank's (max_rows, W, C) strip tensor to rank 0 and un-permute it into an
    (H, W, C) numpy frame on rank 0 (None elsewhere).  `gather_list` may be preallocated."""
    import torch
    import torch.distributed as dist

    if world <= 1:
        return strip[:height].cpu().numpy()
    if rank == 0 and gather_list is None:
        gather_list = [torch.empty_like(strip) for _ in range(world)]
    dist.gather(strip, gather_list=gather_list if rank == 0 else None, dst=0)
    if rank != 0:
        return None
    W, Cc = strip.shape[1], strip.shape[2]
    frame = np.zeros((height, W, Cc), dtype=strip.cpu().numpy().dtype)
    for r in range(world):
        ys = rows_of(height, band_rows, r, world)
        frame[ys] = gather_list[r][:len(ys)].cpu().numpy()
    return frame


def unpermute(strips: List[np.ndarray], height: int, band_rows: int) -> np.ndarray:
    """Host-side inverse of the band assignment for already-gathered strips."""
    world = len(strips)
    W, Cc = strips[0].shape[1], strips[0].shape[2]
    frame = np.zeros((height, W, Cc), strips[0].dtype)
    for r in range(world):
        ys = rows_of(height, band_rows, r, world)
        frame[ys] = strips[r][:len(ys)]
    return frame


def strip_index(height: int, band_rows: int, world: int) -> Optional[np.ndarray]:
    """For each frame row, (rank, row-in-strip): the table rank 0 applies after the gather."""
    out = np.zeros((height, 2), np.int64)
    for r in range(world):
        for k, y in enumerate(rows_of(height, band_rows, r, world)):
            out[y] = (r, k)
    return out
