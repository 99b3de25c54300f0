"""Pixel-tile sharding layout shared by every rank (mirror of csrc/hip/rt_render.hip).

The W x H frame is cut into tile_w x tile_h tiles numbered row-major from the bottom-left
(GL framebuffer order); rank r of `world` owns tiles t with t % world == r (interleaved, so
cheap sky rows and expensive object rows spread evenly).  Each rank keeps its tiles in a
compact buffer [max_local_tiles][tile_h][tile_w] (float4 on the device); rank-major
concatenation of those buffers is what the frame-end gather produces, and `assemble`
un-permutes it exactly like rt_assemble_kernel.
"""
from __future__ import annotations

import numpy as np


def tile_grid(W: int, H: int, tile_w: int, tile_h: int):
    return (W + tile_w - 1) // tile_w, (H + tile_h - 1) // tile_h


def local_tiles(W: int, H: int, tile_w: int, tile_h: int, rank: int, world: int):
    """Global tile ids owned by `rank`, in local order."""
    tx, ty = tile_grid(W, H, tile_w, tile_h)
    return list(range(rank, tx * ty, world))


def max_local_tiles(W: int, H: int, tile_w: int, tile_h: int, world: int) -> int:
    tx, ty = tile_grid(W, H, tile_w, tile_h)
    return (tx * ty + world - 1) // world


def tile_rect(t: int, W: int, H: int, tile_w: int, tile_h: int):
    """(x0, y0, w, h) of global tile t, clipped to the frame."""
    tx, _ = tile_grid(W, H, tile_w, tile_h)
    x0, y0 = (t % tx) * tile_w, (t // tx) * tile_h
    return x0, y0, min(tile_w, W - x0), min(tile_h, H - y0)


def assemble(gathered: np.ndarray, W: int, H: int, tile_w: int, tile_h: int, world: int) -> np.ndarray:
    """gathered: (world, max_local_tiles, tile_h, tile_w, C) -> (H, W, C) frame."""
    tx, _ = tile_grid(W, H, tile_w, tile_h)
    C = gathered.shape[-1]
    out = np.zeros((H, W, C), gathered.dtype)
    for py in range(H):
        ty, ly = divmod(py, tile_h)
        for txi in range(tx):
            gt = ty * tx + txi
            rank, lt = gt % world, gt // world
            x0 = txi * tile_w
            w = min(tile_w, W - x0)
            out[py, x0:x0 + w] = gathered[rank, lt, ly, :w]
    return out
