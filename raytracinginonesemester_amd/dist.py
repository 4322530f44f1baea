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


def gather_p6(strip, height: int, band_rows: int, world: int, rank: int, maxval: int = 255, clamp: bool = True,
              gamma2: bool = True, flip_y: bool = False, stream=None):
    """The frame epilogue on the devices: every rank quantises its float
    strip to P6 samples on its GPU (3 B instead of 12 B per pixel at maxval < 256), one gather of
    the byte strips to rank 0, and rank 0 un-permutes the bands (flipping if asked) on its GPU.
    Returns the P6 file bytes on rank 0, None elsewhere; identical to
    ``encode_p6(gather_frame(...))`` (write_p6, HW1/ppm_p6_lib/src/ppm_p6.cpp:257-301)."""
    import torch
    import torch.distributed as dist

    from . import api

    if not (strip.is_cuda and strip.dtype == torch.float32 and strip.dim() == 3 and strip.shape[2] == 3):
        raise ValueError("gather_p6: expects a (rows, W, 3) float32 device strip")
    strip = strip.contiguous()
    rows, W = strip.shape[0], strip.shape[1]
    bps = 1 if maxval < 256 else 2
    rb = W * 3 * bps
    if stream is None:
        stream = torch.cuda.current_stream(strip.device).cuda_stream
    q = torch.empty((rows, rb), dtype=torch.uint8, device=strip.device)
    api.quantize_p6_device(strip.data_ptr(), W, rows, q.data_ptr(), maxval, clamp, gamma2, False, stream)
    if world > 1:
        on_host = dist.get_backend() == "gloo"
        src = q.cpu() if on_host else q
        buf = torch.empty((world, rows, rb), dtype=torch.uint8, device="cpu" if on_host else strip.device) \
            if rank == 0 else None
        dist.gather(src, gather_list=list(buf.unbind(0)) if rank == 0 else None, dst=0)
        if rank != 0:
            return None
        strips = buf.to(strip.device)
    else:
        strips = q
    frame = torch.empty((height, rb), dtype=torch.uint8, device=strip.device)
    api.unpermute_strips_device(strips.data_ptr(), rows, rb, height, band_rows, max(world, 1), frame.data_ptr(),
                                flip_y, stream)
    return api.p6_header(W, height, maxval) + frame.cpu().numpy().tobytes()


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
