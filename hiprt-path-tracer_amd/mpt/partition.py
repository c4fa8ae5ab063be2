"""Framebuffer row partition across GPUs.

Rank ``k`` of ``n`` owns the interleaved bands ``y // band_height ≡ k (mod n)``; its
framebuffer holds those rows in increasing y ("band-major compact layout", the layout
of ``mpt_get_framebuffer``).  Every pixel's RNG stream depends only on (pixel index,
sample number, seed), so any partition renders the same pixels bit-identically.
"""
from __future__ import annotations

import numpy as np


def rows_of(res_y: int, band_height: int, band_index: int, band_count: int) -> np.ndarray:
    y = np.arange(res_y)
    return y[(y // band_height) % band_count == band_index]


def max_rows(res_y: int, band_height: int, band_count: int) -> int:
    return max(len(rows_of(res_y, band_height, k, band_count)) for k in range(band_count))


def assemble(parts, res_y: int, band_height: int):
    """parts[k]: rank k's compact rows (rows_k[, padding], W, C) -> full (res_y, W, C).
    Works on numpy arrays and torch tensors (the gathered padded buffers)."""
    n = len(parts)
    first = parts[0]
    if hasattr(first, "new_zeros"):          # torch
        out = first.new_zeros((res_y,) + tuple(first.shape[1:]))
        import torch
        for k, p in enumerate(parts):
            ys = rows_of(res_y, band_height, k, n)
            out[torch.as_tensor(ys, device=p.device)] = p[: len(ys)]
        return out
    out = np.zeros((res_y,) + first.shape[1:], first.dtype)
    for k, p in enumerate(parts):
        ys = rows_of(res_y, band_height, k, n)
        out[ys] = p[: len(ys)]
    return out


def gather_frame(local, res_y: int, band_height: int, dist, group=None):
    """Collective gather of every rank's compact rows (torch tensor [rows, W, C]) and
    re-interleave into the full frame on every rank.  With the nccl backend this is one
    RCCL all-gather over xGMI of the padded row buffers; with gloo (CPU tests) the same
    code path runs on host tensors."""
    world = dist.get_world_size(group)
    mr = max_rows(res_y, band_height, world)
    padded = local.new_zeros((mr,) + tuple(local.shape[1:]))
    padded[: local.shape[0]] = local
    parts = [local.new_empty(padded.shape) for _ in range(world)]
    dist.all_gather(parts, padded, group=group)
    return assemble(parts, res_y, band_height)
