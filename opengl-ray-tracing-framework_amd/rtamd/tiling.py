"""Pixel-tile sharding layout shared by every rank (mirror of csrc/hip/rt_render.hip).

The W x H frame is cut into tile_w x tile_h tiles numbered row-major from the bottom-left
(GL framebuffer order).  An owner map assigns every tile to a rank: by default t % world
(interleaved, so cheap sky rows and expensive object rows spread evenly), or `balance` of
measured per-tile costs (rt_tile_costs) for an even split of the work.  Each
rank keeps its tiles, in ascending id, in a compact buffer [max_local_tiles][tile_h][tile_w]
(float4 on the device); rank-major concatenation of those buffers is what the frame-end gather
produces, and `assemble` un-permutes it exactly like rt_assemble_kernel.
"""
from __future__ import annotations

import numpy as np


def tile_grid(W: int, H: int, tile_w: int, tile_h: int):
    return (W + tile_w - 1) // tile_w, (H + tile_h - 1) // tile_h


def modulo_owners(W: int, H: int, tile_w: int, tile_h: int, world: int) -> np.ndarray:
    """rt_resize's default map: tile t -> rank t % world."""
    tx, ty = tile_grid(W, H, tile_w, tile_h)
    return np.arange(tx * ty, dtype=np.int32) % world


def balance(costs, world: int) -> np.ndarray:
    """Owner map from per-tile costs: longest-processing-time-first (tiles by cost descending,
    ties by id; each to the least-loaded rank, ties by rank), so every rank gets within one tile's
    cost of the mean.  Deterministic: every rank computes the same map from the same costs."""
    import heapq
    c = np.asarray(costs, np.int64)
    order = sorted(range(len(c)), key=lambda t: (-int(c[t]), t))
    heap = [(0, r) for r in range(world)]
    owner = np.zeros(len(c), np.int32)
    for t in order:
        load, r = heapq.heappop(heap)
        owner[t] = r
        heapq.heappush(heap, (load + int(c[t]), r))
    return owner


def local_tiles(W: int, H: int, tile_w: int, tile_h: int, rank: int, world: int, owner=None):
    """Global tile ids owned by `rank`, in local order (ascending id)."""
    o = modulo_owners(W, H, tile_w, tile_h, world) if owner is None else np.asarray(owner)
    return [int(t) for t in np.flatnonzero(o == rank)]


def max_local_tiles(W: int, H: int, tile_w: int, tile_h: int, world: int, owner=None) -> int:
    o = modulo_owners(W, H, tile_w, tile_h, world) if owner is None else np.asarray(owner)
    return int(np.bincount(o, minlength=world).max())


def tile_rect(t: int, W: int, H: int, tile_w: int, tile_h: int):
    """(x0, y0, w, h) of global tile t, clipped to the frame."""
    tx, _ = tile_grid(W, H, tile_w, tile_h)
    x0, y0 = (t % tx) * tile_w, (t // tx) * tile_h
    return x0, y0, min(tile_w, W - x0), min(tile_h, H - y0)


def assemble(gathered: np.ndarray, W: int, H: int, tile_w: int, tile_h: int, world: int,
             owner=None) -> np.ndarray:
    """gathered: (world, max_local_tiles, tile_h, tile_w, C) -> (H, W, C) frame."""
    tx, _ = tile_grid(W, H, tile_w, tile_h)
    o = modulo_owners(W, H, tile_w, tile_h, world) if owner is None else np.asarray(owner)
    local = np.zeros(len(o), np.int64)
    seen = np.zeros(world, np.int64)
    for t, r in enumerate(o):
        local[t] = seen[r]
        seen[r] += 1
    C = gathered.shape[-1]
    out = np.zeros((H, W, C), gathered.dtype)
    for py in range(H):
        ty, ly = divmod(py, tile_h)
        for txi in range(tx):
            gt = ty * tx + txi
            rank, lt = int(o[gt]), int(local[gt])
            x0 = txi * tile_w
            w = min(tile_w, W - x0)
            out[py, x0:x0 + w] = gathered[rank, lt, ly, :w]
    return out
