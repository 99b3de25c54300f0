"""A scene whose camera rays land exactly on a shared triangle edge (CPU construction, numpy).

A square quad in the plane z = 0, split along its diagonal x = y into two triangles, seen from
(0, 0, 3) straight down -z by a square frame with a symmetric field of view: for the pixels with
px == py, u == v and the camera direction has d.x == d.y exactly (rt_device.h normalize scales
both components alike), so the hit point has P.x == P.y exactly and the reference's edge function
of the diagonal (RT:273-281) is exactly 0 for both triangles: the strict sign test rejects both,
and the ray goes on to a back wall at z = -1.  The trace kernels' barycentric filter with its
derived margin leaves such points to those edge functions; with the margin forced to 0 it trusts
rows that round to a hair above 0 for one of the triangles (side 3.7; at side 1 they round to 0)
and returns the quad instead.  Every triangle emits its own colour, so the image shows which one
each pixel's camera ray hit.  Encodings: the reference's Triangle_encoded / BVHNode_encoded.
"""
from __future__ import annotations

import numpy as np

from cull_cases import _tri_enc, normalize_f32

HALF_SIDE = 3.7  # (the rows of a quad of half side 1 round to 0 exactly: no contradiction to show)


def diagonal_scene(half_side: float = HALF_SIDE):
    s = float(half_side)
    p = np.array([[-s, -s, 0.0], [s, -s, 0.0], [s, s, 0.0], [-s, s, 0.0]], np.float32)
    w = np.array([[-40.0, -40.0, -1.0], [40.0, -40.0, -1.0], [0.0, 40.0, -1.0]], np.float32)
    tris = [(p[0], p[1], p[2]), (p[0], p[2], p[3]), (w[0], w[1], w[2])]
    tri_enc = np.stack([_tri_enc(*tris[0], (6, 0, 0)), _tri_enc(*tris[1], (0, 6, 0)), _tri_enc(*tris[2], (0, 0, 6))])
    box = [(np.minimum(np.minimum(*q[:2]), q[2]), np.maximum(np.maximum(*q[:2]), q[2])) for q in tris]
    nodes = np.zeros((4, 4, 3), np.float32)
    quad = (np.minimum(box[0][0], box[1][0]), np.maximum(box[0][1], box[1][1]))
    allb = (np.minimum(quad[0], box[2][0]), np.maximum(quad[1], box[2][1]))
    nodes[1] = [(2, 3, 0), (0, 0, 0), allb[0], allb[1]]   # root
    nodes[2] = [(0, 0, 0), (2, 0, 0), quad[0], quad[1]]   # leaf: the two quad triangles
    nodes[3] = [(0, 0, 0), (1, 2, 0), box[2][0], box[2][1]]  # leaf: the wall
    return {"tri_enc": tri_enc, "node_enc": nodes, "tris": tris}


def diagonal_frame_params(W: int):
    """Camera at (0, 0, 3) looking down -z, square frame, half field of view 30 degrees."""
    from rtamd.renderer import FrameParams
    hh = float(np.float32(np.tan(np.radians(30.0))))
    front, right, up = np.array([0, 0, -1], np.float32), np.array([1, 0, 0], np.float32), np.array([0, 1, 0], np.float32)
    lbc = front - np.float32(hh) * right - np.float32(hh) * up
    return FrameParams(position=(0.0, 0.0, 3.0), front=tuple(map(float, front)), right=tuple(map(float, right)),
                       up=tuple(map(float, up)), left_bottom_corner=tuple(map(float, lbc)), half_h=hh, half_w=hh)


def diagonal_camera_rays(W: int):
    """The camera directions of the diagonal pixels (px == py), as rt_device.h computes them."""
    fp = diagonal_frame_params(W)
    lbc, right, up = (np.array(x, np.float32) for x in (fp.left_bottom_corner, fp.right, fp.up))
    hw = hh = np.float32(fp.half_h)
    px = np.arange(W, dtype=np.float32)
    u = (px + np.float32(0.5)) / np.float32(W)
    d = lbc[None] + (u * np.float32(2.0) * hw)[:, None] * right[None] + (u * np.float32(2.0) * hh)[:, None] * up[None]
    return normalize_f32(d.astype(np.float32))
