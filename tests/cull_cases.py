"""Adversarial scenes for the traversal's closest-hit culling (CPU construction, numpy only).

`old_margin_counterexample` searches, with the fp32 restatement of the reference's triangle
test in test_cull_bound.py, for a near-axis-parallel camera ray whose accepted hit on a
triangle T lies several units *before* the entry of T's own bounding box (the computed hit point
is a hair outside the box, and the ray runs almost parallel to the box face it skims).  It then
builds a three-leaf scene in the reference's encodings (Triangle_encoded / BVHNode_encoded,
src/core/Triangle.h:28-39, src/core/BVH.h:17-21): T, a wall BS crossing the ray between T's hit
and T's box entry, and a farther wall F.  The reference tests all three and keeps T (closest);
a traversal that culls T's box once BS is found with the round-1 margin (best + 1e-3 +
1e-3*best) returns BS instead.
"""
from __future__ import annotations

import numpy as np

from test_cull_bound import F, dot, geometric_normal, hit_triangle, slab_entry


def normalize_f32(v):
    """rt_device.h normalize: v * (1 / sqrt(dot(v, v))) in fp32."""
    inv = F(1) / np.sqrt(dot(v, v))
    return v * inv[..., None]


def _slab_exit(S, inv, lo, hi):
    f = (hi - S) * inv
    n = (lo - S) * inv
    return np.min(np.maximum(f, n), axis=-1)


def _material(emissive):
    m = np.zeros((8, 3), np.float32)
    m[0] = emissive                      # emissive
    m[1] = (0.5, 0.5, 0.5)               # baseColor
    m[2] = (0.0, 0.0, 0.5)               # subsurface, metallic, specular
    m[3] = (0.0, 0.5, 0.0)               # specularTint, roughness, anisotropic
    m[5] = (0.0, 1.5, 0.0)               # clearcoatGloss, IOR, transmission
    m[6] = (1.0, 1.0, 1.0)               # mediumColor
    return m


def _tri_enc(p1, p2, p3, emissive):
    t = np.zeros((14, 3), np.float32)
    t[0], t[1], t[2] = p1, p2, p3
    n = np.cross((p2 - p1).astype(np.float64), (p3 - p1).astype(np.float64))
    n = (n / np.linalg.norm(n)).astype(np.float32)
    t[3] = t[4] = t[5] = n
    t[6:14] = _material(emissive)
    return t


def _wall(S, d, t_w, axis):
    """A triangle in the plane x_axis = const crossing the ray at parameter ~t_w."""
    c = (S.astype(np.float64) + d.astype(np.float64) * t_w)
    o = [a for a in range(3) if a != axis]
    p = np.tile(c, (3, 1))
    p[0, o[0]] -= 1.0; p[0, o[1]] -= 1.0
    p[1, o[0]] += 2.0; p[1, o[1]] -= 1.0
    p[2, o[0]] -= 1.0; p[2, o[1]] += 2.0
    return [x.astype(np.float32) for x in p]


def old_margin_counterexample(seed: int = 0, batch: int = 50_000, tries: int = 40):
    rng = np.random.default_rng(seed)
    for _ in range(tries):
        n = batch
        # the computed hit point leaves the box only near the triangle's extreme vertex along some
        # axis b; a ray almost parallel to another axis a then skims face b for a long stretch
        scale = rng.choice([0.05, 1.0, 8.0], size=(n, 1))
        centre = rng.uniform(-48, 48, size=(n, 3))
        P3 = centre[:, None, :] + rng.normal(size=(n, 3, 3)) * scale[:, None, :]
        a = rng.integers(0, 3, size=n)
        b = (a + rng.integers(1, 3, size=n)) % 3
        sgn = rng.choice([-1, 1], size=n)
        vi = np.argmax(P3[np.arange(n), :, b] * sgn[:, None], axis=1)
        w = np.abs(rng.normal(size=(n, 3))) * 10.0 ** rng.uniform(-8, -5, size=(n, 1))
        w[np.arange(n), vi] = 1.0 - (w.sum(1) - w[np.arange(n), vi])
        target = (w[:, :, None] * P3).sum(1)
        p1, p2, p3 = P3[:, 0], P3[:, 1], P3[:, 2]
        lbc = np.zeros((n, 3))
        lbc[np.arange(n), a] = rng.choice([-1, 1], size=n)
        lbc += rng.normal(size=(n, 3)) * 10.0 ** rng.uniform(-7, -5, size=(n, 1))
        lbc = (lbc / np.linalg.norm(lbc, axis=1, keepdims=True)).astype(np.float32)
        d = normalize_f32(lbc)
        t_aim = rng.uniform(5.0, 40.0, size=(n, 1))
        S = (target - d.astype(np.float64) * t_aim).astype(np.float32)
        p1, p2, p3 = (x.astype(np.float32) for x in (p1, p2, p3))
        N = geometric_normal(p1, p2, p3)
        ok, t = hit_triangle(p1, p2, p3, N, S, d)
        lo = np.minimum(np.minimum(p1, p2), p3)
        hi = np.maximum(np.maximum(p1, p2), p3)
        with np.errstate(all="ignore"):
            inv = F(1) / d
            t0 = slab_entry(S, inv, lo, hi)
            t1 = _slab_exit(S, inv, lo, hi)
        tt = t.astype(np.float64)
        gap = t0.astype(np.float64) - tt
        viol = ok & (t1 >= t0) & (t0 > 0) & np.isfinite(inv).all(1) & (gap > 0.5 + 2e-3 * tt + 1e-2 * t0)
        if not viol.any():
            continue
        i = int(np.argmax(np.where(viol, gap, -1.0)))
        ax = int(np.argmax(np.abs(d[i])))
        t_c, t_e = float(tt[i]), float(t0[i])
        walls = [_wall(S[i], d[i], t_c + f * (t_e - t_c), ax) for f in (0.3, 0.6)]
        tris = [(p1[i], p2[i], p3[i])] + walls
        # every wall must be hit where intended, in front of T's box entry
        hits = []
        for q in tris:
            qq = [x[None] for x in q]
            okq, tq = hit_triangle(*qq, geometric_normal(*qq), S[i][None], d[i][None])
            hits.append((bool(okq[0]), float(tq[0])))
        if not all(h[0] for h in hits) or not (hits[0][1] < hits[1][1] < hits[2][1] < t_e):
            continue
        tri_enc = np.stack([_tri_enc(*tris[0], (8, 0, 0)), _tri_enc(*tris[1], (0, 8, 0)),
                            _tri_enc(*tris[2], (0, 0, 8))])
        box = [(np.minimum(np.minimum(*q[:2]), q[2]), np.maximum(np.maximum(*q[:2]), q[2])) for q in tris]
        nodes = np.zeros((6, 4, 3), np.float32)

        def node(j, left, right, nn, index, b):
            nodes[j, 0] = (left, right, 0)
            nodes[j, 1] = (nn, index, 0)
            nodes[j, 2], nodes[j, 3] = b

        def union(*bs):
            return (np.min([b[0] for b in bs], 0), np.max([b[1] for b in bs], 0))

        node(1, 2, 5, 0, 0, union(*box))
        node(2, 3, 4, 0, 0, union(box[1], box[2]))
        node(3, 0, 0, 1, 1, box[1])   # BS
        node(4, 0, 0, 1, 2, box[2])   # F
        node(5, 0, 0, 1, 0, box[0])   # T
        return {"tri_enc": tri_enc, "node_enc": nodes, "position": S[i].copy(), "lbc": lbc[i].copy(),
                "direction": d[i].copy(), "t_hit": hits[0][1], "t_wall": hits[1][1], "t0_box": t_e}
    raise RuntimeError("no counterexample found")
