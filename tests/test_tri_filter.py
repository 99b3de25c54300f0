"""CPU: the trace kernels' barycentric edge filter never contradicts the reference's edge test.

wf_trace decides "hit point inside the triangle" with two barycentric rows (R2, R3 of the traversal
record, csrc/common/tri_filter.h) and runs the reference's three fp32 edge functions
(RT:273-281) only when min(b) lies within the margin m = k1 * max|P - p1| * (max|R2| + max|R3|) + k0.
This test restates both computations in numpy fp32 (the kernel's operation order; its fma emulated
through float64) on the C3 mesh's triangles and on adversarial ones (slivers, far from the origin,
tiny), with points placed on edges, at vertices, off the plane and at random, and checks:
  * wherever the filter is decisive, its answer equals the reference's edge test;
  * the filter is decisive for almost every point not within a hair of an edge;
  * with the margin forced to 0 it does contradict the reference on the on-edge points (so the
    points really probe the margin: the negative control).
The GPU side of the same decision is covered bit for bit by the image parity tests.
"""
import numpy as np
import pytest

from rtamd import configs as cf
from rtamd import scene_lib as sl

f32 = np.float32


def _normal(p1, p2, p3):
    """rt_render.hip geometric_normal: the reference's N = normalize(cross(p2-p1, p3-p1)) in fp32
    (NaN for a degenerate triangle)."""
    a, b = p2 - p1, p3 - p1
    c = np.stack([a[:, 1] * b[:, 2] - b[:, 1] * a[:, 2], a[:, 2] * b[:, 0] - b[:, 2] * a[:, 0],
                  a[:, 0] * b[:, 1] - b[:, 0] * a[:, 1]], 1)
    with np.errstate(all="ignore"):
        inv = f32(1) / np.sqrt((c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]) + c[:, 2] * c[:, 2])
        return c * inv[:, None]


def _tri_records(p1, p2, p3):
    n = _normal(p1, p2, p3)
    tri = np.zeros((len(p1), 3, 4), f32)
    tri[:, 0, :3], tri[:, 1, :3], tri[:, 2, :3] = p1, p2, p3
    tri[:, :, 3] = n
    return tri


def _cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - b[..., 1] * a[..., 2], a[..., 2] * b[..., 0] - b[..., 2] * a[..., 0],
                     a[..., 0] * b[..., 1] - b[..., 0] * a[..., 1]], -1)


def _dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def exact_inside(tri, P):
    """The reference's edge test (RT:273-281) in fp32, operation for operation."""
    p1, p2, p3, N = tri[:, 0, :3], tri[:, 1, :3], tri[:, 2, :3], tri[:, :, 3]
    with np.errstate(all="ignore"):
        e1 = _dot(_cross(p2 - p1, P - p1), N)
        e2 = _dot(_cross(p3 - p2, P - p2), N)
        e3 = _dot(_cross(p1 - p3, P - p3), N)
    return ((e1 > 0) & (e2 > 0) & (e3 > 0)) | ((e1 < 0) & (e2 < 0) & (e3 < 0))


def _fma(a, b, c):
    """fp32 fmaf(a, b, c) correctly rounded (rounding a*b + c to float64 and then to
    float32 rounds twice).  The float64 product of two floats is exact; the float64 sum is rounded
    to odd (TwoSum gives its exact error; an inexact sum with an even last bit moves one ulp toward
    the exact value), and a round-to-odd result with 29 extra bits rounds to the float32 nearest the
    exact a*b + c (Boldo & Melquiond)."""
    p = a.astype(np.float64) * b.astype(np.float64)
    c = np.broadcast_to(c, p.shape).astype(np.float64)
    s = p + c
    bb = s - p
    err = (p - (s - bb)) + (c - bb)
    bits = s.view(np.int64).copy()
    fix = (err != 0) & ((bits & 1) == 0)
    up = (err > 0) == (s > 0)  # the exact value lies away from zero
    bits[fix] += np.where(up[fix], 1, -1)
    return bits.view(np.float64).astype(f32)


def test_fma_restatement_rounds_once():
    """_fma against exact rational arithmetic, including cases built so that the float64 sum lands
    on a float32 rounding midpoint (where rounding twice goes wrong)."""
    from fractions import Fraction
    rng = np.random.default_rng(5)
    a = rng.uniform(-4, 4, 2000).astype(f32)
    b = rng.uniform(-4, 4, 2000).astype(f32)
    c = rng.uniform(-4, 4, 2000).astype(f32)
    # midpoint cases: c = -(a*b) rounded, plus a tiny term, so the exact value sits next to a tie
    half_ulp = f32(2.0) ** -25
    a2 = np.array([1 + 2 ** -23, 1 + 3 * 2 ** -23, 3.0, 1 + 2 ** -12], f32)
    b2 = np.array([1 + 2 ** -23, 1 - 2 ** -23, 1 + 2 ** -22, 1 + 2 ** -12], f32)
    c2 = np.array([half_ulp, -half_ulp, f32(2.0 ** -24), f32(-2.0 ** -30)], f32)
    A, B, Cc = (np.concatenate(x) for x in ((a, a2), (b, b2), (c, c2)))
    got = _fma(A, B, Cc)
    for x, y, z, g in zip(A, B, Cc, got):
        exact = Fraction(float(x)) * Fraction(float(y)) + Fraction(float(z))
        lo = f32(float(exact))
        cands = [lo, np.nextafter(lo, f32(np.inf)), np.nextafter(lo, f32(-np.inf))]
        best = min(cands, key=lambda v: (abs(Fraction(float(v)) - exact), int(np.asarray(v).view(np.uint32)) & 1))
        assert g == best, (x, y, z, g, best)


def filter_decision(rec, P, k1, k0):
    """rt_wavefront.h tl_triangle_calc's filter: (decisive, inside)."""
    p1, R2, R3 = rec[:, 0, :3], rec[:, 1, :3], rec[:, 2, :3]
    q = (P - p1).astype(f32)
    b2 = _fma(R2[:, 0], q[:, 0], _fma(R2[:, 1], q[:, 1], R2[:, 2] * q[:, 2]))
    b3 = _fma(R3[:, 0], q[:, 0], _fma(R3[:, 1], q[:, 1], R3[:, 2] * q[:, 2]))
    b1 = (f32(1) - b2) - b3
    mn = np.minimum(b1, np.minimum(b2, b3))
    dq = np.abs(q).max(1)
    lr = np.abs(R2).max(1) + np.abs(R3).max(1)
    m = (dq * lr) * f32(k1) + f32(k0)
    decisive = (np.abs(mn) > m) & (m < f32(0.25))
    return decisive, mn > 0


def _points(tri, rng):
    """Probe points per triangle: on each edge, near each vertex, off the plane, at random."""
    p = [tri[:, k, :3].astype(np.float64) for k in range(3)]
    N = tri[:, :, 3].astype(np.float64)
    scale = np.maximum.reduce([np.abs(p[1] - p[0]).max(1), np.abs(p[2] - p[1]).max(1), np.abs(p[0] - p[2]).max(1)])
    out = {}
    on = []
    for a, b in ((0, 1), (1, 2), (2, 0)):
        s = rng.uniform(-0.05, 1.05, len(scale))[:, None]
        on.append((p[a] + s * (p[b] - p[a])).astype(f32))  # on the edge's line, within rounding
    out["on_edge"] = on
    out["near_vertex"] = [(p[k] + (rng.normal(size=p[k].shape) * scale[:, None] * 1e-6)).astype(f32) for k in range(3)]
    w = rng.uniform(-0.2, 1.2, (len(scale), 2))
    inplane = p[0] + w[:, :1] * (p[1] - p[0]) + w[:, 1:] * (p[2] - p[0])
    out["random"] = [inplane.astype(f32)]
    out["off_plane"] = [(inplane + N * (scale * h)[:, None]).astype(f32) for h in (1e-6, 1e-3, 0.3)]
    return out


def _adversarial(rng):
    """Slivers, triangles far from the origin and tiny ones."""
    base = rng.uniform(-1, 1, (400, 3, 3))
    sl_ = base.copy()
    sl_[:, 2] = sl_[:, 0] + (sl_[:, 1] - sl_[:, 0]) * 0.5 + rng.normal(size=(400, 3)) * 1e-3  # aspect ~1e3
    far = base * 0.01 + np.array([1000.0, -500.0, 250.0])
    tiny = base * 1e-4 + 0.3
    return np.concatenate([base, sl_, far, tiny]).astype(f32)


def _check(tri, rng, label):
    rec, k1, k0, flagged = sl.tri_filter(tri)
    assert np.array_equal(rec[:, :, 3], tri[:, :, 3]) and np.array_equal(rec[:, 0, :3], tri[:, 0, :3])
    stats = {}
    for kind, sets in _points(tri, rng).items():
        for P in sets:
            ok = np.isfinite(tri[:, :, 3]).all(1)
            dec, ins = filter_decision(rec, P, k1, k0)
            ex = exact_inside(tri, P)
            bad = ok & dec & (ins != ex)
            assert not bad.any(), f"{label}/{kind}: filter contradicts the edge test on {bad.sum()} points"
            d, n = stats.get(kind, (0, 0))
            stats[kind] = (d + int((dec & ok).sum()), n + int(ok.sum()))
    return stats, (k1, k0, flagged)


def test_filter_agrees_with_reference_edges_on_c3_mesh():
    rng = np.random.default_rng(7)
    s = cf.config_scene("C3").soa
    idx = rng.choice(len(s["p1"]), 20000, replace=False)
    tri = _tri_records(s["p1"][idx].astype(f32), s["p2"][idx].astype(f32), s["p3"][idx].astype(f32))
    stats, (k1, k0, flagged) = _check(tri, rng, "C3")
    assert 0 < k1 < 1e-4 and 0 < k0 < 1e-3, (k1, k0)
    assert flagged <= 0.002 * len(tri) + 1
    # decisive for nearly all points away from the edges; the on-edge probes mostly fall back
    for kind in ("random", "off_plane"):
        d, n = stats[kind]
        assert d / n > 0.99, (kind, d / n)
    d, n = stats["on_edge"]
    assert d / n < 0.2, d / n


def test_filter_agrees_with_reference_edges_on_adversarial_triangles():
    rng = np.random.default_rng(11)
    a = _adversarial(rng)
    tri = _tri_records(a[:, 0], a[:, 1], a[:, 2])
    stats, (k1, k0, flagged) = _check(tri, rng, "adversarial")
    assert flagged >= 400  # the slivers are left to the reference's test ...
    assert k0 < 1e-3  # ... and the margin stays that of the well-shaped triangles
    d, n = stats["random"]
    assert d / n > 0.7, d / n  # (points on the 400 slivers are never decisive)


def test_zero_margin_contradicts_reference_on_edges():
    """Negative control: the on-edge probes do reach the decision boundary."""
    rng = np.random.default_rng(3)
    s = cf.config_scene("C3").soa
    idx = rng.choice(len(s["p1"]), 20000, replace=False)
    tri = _tri_records(s["p1"][idx].astype(f32), s["p2"][idx].astype(f32), s["p3"][idx].astype(f32))
    rec, _, _, _ = sl.tri_filter(tri)
    wrong = 0
    for P in _points(tri, rng)["on_edge"]:
        dec, ins = filter_decision(rec, P, 0.0, 0.0)
        wrong += int((dec & (ins != exact_inside(tri, P))).sum())
    assert wrong > 0


def test_empty_and_degenerate_triangles():
    out, k1, k0, flagged = sl.tri_filter(np.zeros((0, 3, 4), f32))
    assert out.shape == (0, 3, 4) and k0 > 0
    p = np.array([[0, 0, 0], [1, 1, 1], [2, 2, 2]], f32)[None]  # collinear: N is NaN, never reaches the edges
    tri = _tri_records(p[:, 0], p[:, 1], p[:, 2])
    out, _, _, flagged = sl.tri_filter(tri)
    assert flagged == 1 and not out[:, 1:, :3].any()


def test_diagonal_scene_probes_the_margin():
    """tests/edge_cases.py: the camera rays of the diagonal pixels hit the shared edge exactly.  The
    reference's edge test rejects both triangles there; the filter with the derived margin is never
    decisive against it, and with the margin forced to 0 it contradicts it for most of those pixels
    (the scene tests/test_gpu_tri_filter.py renders as the GPU negative control)."""
    from edge_cases import diagonal_camera_rays, diagonal_scene
    from test_cull_bound import geometric_normal, hit_triangle
    sc = diagonal_scene()
    W = 128
    d = diagonal_camera_rays(W)
    assert np.array_equal(d[:, 0], d[:, 1])
    S = np.tile(np.array([0, 0, 3], f32), (W, 1))
    p1, p2, p3 = (np.stack([t[k] for t in sc["tris"][:2]]) for k in range(3))
    tri = _tri_records(p1, p2, p3)
    rec, k1, k0, _ = sl.tri_filter(tri)
    wrong = 0
    for k in range(2):
        q = [np.repeat(x[k:k + 1], W, 0) for x in (p1, p2, p3)]
        ok, t = hit_triangle(*q, geometric_normal(*q), S, d)
        assert not ok.any()  # the reference: neither triangle (the edge function is exactly 0)
        P = (S + d * t[:, None]).astype(f32)
        assert np.array_equal(P[:, 0], P[:, 1])
        r = np.repeat(rec[k:k + 1], W, 0)
        dec, ins = filter_decision(r, P, k1, k0)
        assert not (dec & ins).any()
        dec0, ins0 = filter_decision(r, P, 0.0, 0.0)
        wrong += int((dec0 & ins0).sum())
    assert wrong > W // 2, wrong
