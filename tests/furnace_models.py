"""Expected values of the reference's BSDF integrator for furnace scenes the plane furnace
(tests/test_furnace.py) does not reach, evaluated in numpy from the GLSL's formulas alone: no
sampling routine of either implementation enters them.  Test infrastructure only.

* A glass slab (two parallel copies of the reference's floor quad, roughness 0 so that
  m.ax = m.ay = 0.001, transmission 1, metallic 0) in a constant environment, with an ABSORB or
  EMISSIVE medium.  Every camera ray hits the top face; from there a path is a chain of
  reflect / refract choices at the two faces, each with the reference's probabilities and
  weights (fragment_shader_ray_tracing.glsl, "RT:"):
    - DisneySample picks reflection when xi_3 < F, F = DielectricFresnel(|V.H|, eta) (RT:1136-1155,
      metallic 0: R7's uninitialised L drops out), with H the VNDF normal, = N here;
    - eta = 1 / IOR at every face, entering or leaving, since N is flipped towards V before
      DisneyEval / DisneySample test V.N (R10, RT:1010, RT:1079);
    - a reflection multiplies history by f / pdf = Fs G1(L) / F with Fs = mix(F0^2, 1, F)
      (EvalSpecReflection over its pdf times the lobe probability F, RT:950-964, RT:1150-1153);
    - a refraction does NOT multiply by f / pdf (R9, RT:1429-1431); the medium acts instead:
      ABSORB history *= exp(-(1 - color) * hit.distance * density), EMISSIVE
      Lo += color * hit.distance * density * history, where hit.distance is the segment that
      ARRIVED at the face (R11, RT:1434-1439): for the camera's first hit the camera-to-glass
      distance, inside the slab the face-to-face segment;
    - a ray that escapes adds history * Le * f_eval / pdf_eval of the full DisneyEval at the
      sampled direction (RT:1483-1497, the second application of the weight, R9): G1(L) (Fs + 1 - F)
      after a reflection, G1(L) eta^2 (Fs + 1 - F) after a refraction (EvalSpecRefraction's eta^2
      and (1 - F) over its pdf and the refraction lobe weight, RT:966-984, RT:537-550), with MIS
      weight 1 (the delta lobe's pdf ~ 1 / (pi a^2) dwarfs the map's);
    - maxBounce interactions at most (RT:1374): the ray sampled at the last one still escapes;
    - next-event estimation: shadow rays from inside the slab hit the other face; from the top
      face's outside only the tails of the 0.001-wide reflection lobe count, and MIS moves the
      same tails' weight off the escaping sample (`nee_tail`: the net of both, ~1e-5 of Le).
* The BSDF integrator's clearcoat with R23: EvalClearcoat evaluates GTR1 with alpha =
  clearcoatGloss itself (RT:994) while SampleGTR1(rgh, r1, r2) (RT:716-729) draws
  cos(theta_h) AND phi_h from r1 alone: the sampled half vectors lie on a curve, and the
  estimator's expectation over that lobe is a 1-D integral over r1 (`clearcoat_curve_term`).
"""
from __future__ import annotations

from functools import lru_cache

import numpy as np

A_SMOOTH = 0.001        # m.ax = m.ay = max(0.001, roughness^2) at roughness 0 (RT:205-207)


def dielectric_fresnel(c, eta):
    """DielectricFresnel(cosThetaI, eta) (RT:487-500), fp64."""
    c = np.asarray(c, np.float64)
    s2 = eta * eta * (1.0 - c * c)
    ct = np.sqrt(np.maximum(1.0 - s2, 0.0))
    rs = (eta * ct - c) / (eta * ct + c)
    rp = (eta * c - ct) / (eta * c + ct)
    return np.where(s2 > 1.0, 1.0, 0.5 * (rs * rs + rp * rp))


def smith_g1(wz, wxy2, a):
    """SmithG_GGX_Aniso with ax = ay = a (RT:466-471)."""
    return 2.0 * wz / (wz + np.sqrt(a * a * wxy2 + wz * wz))


def camera_rays(fp, W, H):
    """Unit camera-ray directions (H, W, 3), rows bottom-up as the accumulation stores them
    (RT:1520-1527: normalize(LBC + 2u halfW right + 2v halfH up), u = (px + .5) / W)."""
    lbc, right, up = (np.asarray(x, np.float64) for x in (fp.left_bottom_corner, fp.right, fp.up))
    u = (np.arange(W) + 0.5) / W
    v = (np.arange(H) + 0.5) / H
    d = (lbc[None, None, :] + (u[None, :, None] * 2 * fp.half_w) * right[None, None, :]
         + (v[:, None, None] * 2 * fp.half_h) * up[None, None, :])
    return d / np.linalg.norm(d, axis=-1, keepdims=True)


@lru_cache(maxsize=None)
def _nee_tail_table(eta: float, n_mu: int = 24):
    """What the MIS split adds to the delta-lobe model at a face seen from its open side, in
    units of Le: the light sample's term (RT:1380-1405) int w_l f cos dw, minus the share w_l of
    the escaping BSDF sample that the model counts at full weight, int w_l f cos (f_e cos / p_e)
    dw with f_e cos / p_e = G1(L) (Fs + 1 - F) (RT:1483-1497); over the reflection lobe's
    hemisphere in half-vector polar coordinates around N (log-spaced near the peak), constant-map
    hdrPdf 1 / (2 pi^2 sin theta) with the map's pole along N.  (The refraction lobe's tails lose
    a similar ~1e-4 of their weight to w_l; not modelled.)"""
    a = A_SMOOTH
    f0 = ((1.0 - eta) / (1.0 + eta)) ** 2
    th = np.concatenate([np.geomspace(1e-6, 0.05, 500), np.linspace(0.05, np.pi / 2, 400)[1:]])
    dth = np.gradient(th)
    nph = 180
    ph = (np.arange(nph) + 0.5) * 2 * np.pi / nph
    T, P = np.meshgrid(th, ph, indexing="ij")
    Hh = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1)
    dwH = np.sin(T) * dth[:, None] * (2 * np.pi / nph)
    D = a * a / (np.pi * ((a * a - 1) * Hh[..., 2] ** 2 + 1) ** 2)
    mus = np.linspace(0.02, 1.0, n_mu)
    out = []
    for mu in mus:
        V = np.array([np.sqrt(1 - mu * mu), 0.0, mu])
        VH = Hh @ V
        L = 2 * VH[..., None] * Hh - V
        ok = (L[..., 2] > 0) & (VH > 0)
        F = dielectric_fresnel(np.abs(VH), eta)
        Fs = f0 + (1 - f0) * F
        g1v = smith_g1(mu, 1 - mu * mu, a)
        g1l = smith_g1(np.abs(L[..., 2]), L[..., 0] ** 2 + L[..., 1] ** 2, a)
        fcos = Fs * D * g1v * g1l / (4 * mu)
        pb = g1v * D / (4 * mu) * Fs / (Fs + 1 - F)           # pdf x specReflectWt (RT:1053-1057)
        pl = 1.0 / (2 * np.pi ** 2 * np.maximum(np.sqrt(np.maximum(0, 1 - L[..., 2] ** 2)), 1e-10))
        wl = pl ** 2 / (pl ** 2 + pb ** 2)
        out.append(float(np.sum(np.where(ok, wl * fcos * (1.0 - g1l * (Fs + 1 - F)) * 4 * np.abs(VH) * dwH, 0.0))))
    return mus, np.array(out)


def nee_tail(mu, eta):
    mus, tab = _nee_tail_table(float(eta))
    return np.interp(mu, mus, tab)


def slab_expectation(dirs, cam, y_top: float, thickness: float, ior: float, medium: str, color, density: float,
                     le: float, max_bounce: int = 8, variant: str = ""):
    """Per camera ray: the expected pixel (RGB) of the reference BSDF integrator for the glass
    slab described in the module docstring, camera at `cam`, faces at y_top and y_top - thickness,
    environment radiance `le` (= map value x envIntensity).  Returns (expected (..., 3), the
    horizontal travel of the deepest path from the first hit, per ray).
    variant (what a test must be able to tell apart): "r11_physical" = the medium acts only over
    the segments inside the glass (the camera segment is not absorbed / does not emit);
    "r9_weighted" = refractions multiply history by their f / pdf (G1(L) eta^2) like reflections."""
    eta = 1.0 / ior
    f0 = ((1.0 - eta) / (1.0 + eta)) ** 2
    color = np.asarray(color, np.float64)
    mu0 = -dirs[..., 1]
    t0 = (y_top - cam[1]) / dirs[..., 1]
    d0 = t0 - 1e-5                                     # hit.distance = t - 0.00001 (RT:284)
    sin0 = np.sqrt(np.maximum(0.0, 1.0 - mu0 * mu0))
    sin_in = eta * sin0
    mu_in = np.sqrt(1.0 - sin_in * sin_in)
    sin_out = eta * sin_in                             # leaving with eta = 1 / IOR again (R10)
    mu_out = np.sqrt(1.0 - sin_out * sin_out)
    seg = thickness / mu_in                            # face-to-face segment inside the slab
    a = A_SMOOTH

    def g1(mu):
        return smith_g1(mu, 1.0 - mu * mu, a)

    def F(mu):
        return dielectric_fresnel(mu, eta)

    def Fs(mu):
        return f0 + (1.0 - f0) * F(mu)

    def medium_on_refraction(hist, dist):
        """(history after, emission added) for a refraction after a segment of length dist"""
        if variant == "r9_weighted":
            hist = hist * eta * eta
        if medium == "absorb":
            return hist * np.exp(-(1.0 - color) * dist[..., None] * density), 0.0
        if medium == "emissive":
            return hist, color * dist[..., None] * density * hist
        return hist, 0.0

    shape = mu0.shape + (3,)
    total = np.zeros(shape)
    # bounce 0: the top face from outside, reached by the camera ray (segment d0)
    total += le * nee_tail(mu0, eta)[..., None]
    p = F(mu0)[..., None]
    w_refl = (Fs(mu0) * g1(mu0) / F(mu0))[..., None]                  # history *= f / pdf
    total += le * p * w_refl * (g1(mu0) * (Fs(mu0) + 1.0 - F(mu0)))[..., None]   # escapes upwards
    hist, emit = medium_on_refraction(np.ones(shape), 0.0 * d0 if variant == "r11_physical" else d0)
    total += (1.0 - p) * emit
    # inside: a ray at mu_in reaches the other face after `seg`; paths carry their probability
    prob = (1.0 - p) * np.ones(shape)
    for bounce in range(1, max_bounce):
        pr = F(mu_in)[..., None]
        # refract out of the slab (segment seg absorbed / emitting), escape below or above
        h_out, emit = medium_on_refraction(hist, seg)
        total += prob * (1.0 - pr) * (emit + le * h_out * (g1(mu_out) * eta * eta * (Fs(mu_in) + 1.0 - F(mu_in)))[..., None])
        # reflect inside: history *= Fs G1 / F, next face
        hist = hist * (Fs(mu_in) * g1(mu_in) / F(mu_in))[..., None]
        prob = prob * pr
    # (the ray reflected at the last interaction reaches a face after maxBounce: the loop ends)
    travel = (max_bounce + 1) * thickness * sin_in / mu_in
    return total, travel


# ------------------------------------------------------------------ BSDF clearcoat (R23)
def disney_eval_nonmetal(V, L, roughness: float, ior: float, clearcoat: float, gloss: float, base: float = 1.0):
    """DisneyEval (RT:1002-1067) of a non-metal, transmission 0, grey base colour `base`,
    specularTint / sheen / subsurface 0, in the local frame (N = +z): f * |L.z| and the
    lobe-weighted pdf.  (base 0 with IOR 1 leaves the clearcoat lobe alone: diffuse weight
    (1 - metallic)(1 - transmission) Luminance(base) = 0, specCol = F0^2 = 0 and the dielectric
    Fresnel at eta = 1 is 0.)"""
    eta = 1.0 / ior
    f0 = ((1.0 - eta) / (1.0 + eta)) ** 2
    a = max(1e-3, roughness * roughness)
    Hh = L + V
    Hh = Hh / np.linalg.norm(Hh, axis=-1, keepdims=True)
    LdotH = np.sum(L * Hh, axis=-1)
    VdotH = np.sum(V * Hh, axis=-1)
    Lz, Vz = L[..., 2], V[..., 2]
    F = dielectric_fresnel(np.abs(VdotH), eta)
    Fs = f0 + (1 - f0) * F
    rsum = base + Fs + 0.25 * clearcoat
    wd, ws, wc = base / rsum, Fs / rsum, 0.25 * clearcoat / rsum

    def schlick(u):
        return np.clip(1.0 - u, 0.0, 1.0) ** 5
    fd90 = 0.5 + 2.0 * LdotH * LdotH * roughness
    Fd = (1 + (fd90 - 1) * schlick(Lz)) * (1 + (fd90 - 1) * schlick(Vz))
    f = base * Fd / np.pi
    pdf = wd * Lz / np.pi
    D = 1.0 / (np.pi * a * a * ((Hh[..., 0] / a) ** 2 + (Hh[..., 1] / a) ** 2 + Hh[..., 2] ** 2) ** 2)
    g1v = smith_g1(Vz, V[..., 0] ** 2 + V[..., 1] ** 2, a)
    g1l = smith_g1(np.abs(Lz), L[..., 0] ** 2 + L[..., 1] ** 2, a)
    f = f + Fs * D * g1v * g1l / (4 * Lz * Vz)
    pdf = pdf + ws * g1v * D / (4 * Vz)
    if clearcoat > 0:
        Dc = gtr1(Hh[..., 2], gloss)
        Fc = 0.04 + 0.96 * dielectric_fresnel(VdotH, 1.0 / 1.5)
        Gc = smith_g_ggx(Lz, 0.25) * smith_g_ggx(Vz, 0.25)
        f = f + 0.25 * clearcoat * Fc * Dc * Gc / (4 * Lz * Vz)
        pdf = pdf + wc * Dc * Hh[..., 2] / (4 * VdotH)
    ok = (Lz > 0) & (Vz > 0)
    return np.where(ok, f * np.abs(Lz), 0.0), np.where(ok, pdf, 0.0)


def gtr1(c, alpha):
    """GTR1(NdotH, alpha) (RT:431-437)."""
    if alpha >= 1.0:
        return np.full_like(np.asarray(c, np.float64), 1.0 / np.pi)
    a2 = alpha * alpha
    return (a2 - 1) / (np.pi * np.log(a2) * (1 + (a2 - 1) * c * c))


def smith_g_ggx(ndotv, alpha_g):
    """SmithG_GGX(NdotV, alphaG) (RT:456-462)."""
    a = alpha_g * alpha_g
    b = ndotv * ndotv
    return 2.0 * ndotv / (ndotv + np.sqrt(a + b - a * b))


def clearcoat_curve_term(V, roughness: float, ior: float, clearcoat: float, gloss: float, n: int = 4096,
                         base: float = 1.0):
    """The clearcoat lobe's share of the escaping BSDF sample's expectation, in units of Le: the
    lobe is picked with DisneySample's approxFresnel weight and history divides by that same
    weight, so the share is E_r[(f_cc cos / pdf_cc)(L(r)) * w_b(L(r)) * (f_eval / pdf_eval)(L(r))]
    over r uniform on [0, 1), with L(r) = reflect(-V, H(r)), H(r) = SampleGTR1(gloss, r, .) whose
    theta AND phi both come from r (R23, RT:716-729).  f_cc cos / pdf_cc =
    0.25 cc F G (V.H) / (V.z H.z) (EvalClearcoat's D cancels, RT:986-1000).  V: local (3,) unit."""
    r = (np.arange(n) + 0.5) / n
    a = max(0.001, gloss)
    a2 = a * a
    phi = r * 2 * np.pi
    cos_t = np.sqrt((1.0 - a2 ** (1.0 - r)) / (1.0 - a2))
    sin_t = np.clip(np.sqrt(1.0 - cos_t * cos_t), 0.0, 1.0)
    Hh = np.stack([sin_t * np.cos(phi), sin_t * np.sin(phi), cos_t], -1)
    VH = Hh @ V
    L = 2 * VH[:, None] * Hh - V
    L = L / np.linalg.norm(L, axis=-1, keepdims=True)
    ok = L[:, 2] > 0                                  # else EvalClearcoat's pdf is 0: the path ends
    Vz = V[2]
    Fc = 0.04 + 0.96 * dielectric_fresnel(VH, 1.0 / 1.5)
    Gc = smith_g_ggx(np.abs(L[:, 2]), 0.25) * smith_g_ggx(Vz, 0.25)
    w_hist = 0.25 * clearcoat * Fc * Gc * VH / (Vz * Hh[:, 2])
    fe, pe = disney_eval_nonmetal(np.broadcast_to(V, L.shape), L, roughness, ior, clearcoat, gloss, base)
    pl = 1.0 / (2 * np.pi ** 2 * np.maximum(np.sqrt(np.maximum(0, 1 - L[:, 2] ** 2)), 1e-10))
    wb = pe ** 2 / (pe ** 2 + pl ** 2)
    val = np.where(ok & (pe > 0), w_hist * wb * fe / np.where(pe > 0, pe, 1.0), 0.0)
    return float(val.mean())


def bsdf_clearcoat_other_terms(mu: float, roughness: float, ior: float, clearcoat: float, gloss: float,
                               nth: int = 200, nph: int = 400, base: float = 1.0):
    """The light sample (A, RT:1380-1405) and the diffuse + specular lobes' share of the escaping
    BSDF sample (B) for the same material, isotropic in V's azimuth: A = int w_l f_eval cos dw,
    B = int (f_d + f_s) cos w_b f_eval cos / pdf_eval dw (those lobes sample their eval pdfs, so
    the lobe weights cancel as in tests/test_furnace.py), in units of Le."""
    th = (np.arange(nth) + 0.5) * (np.pi / 2) / nth
    ph = (np.arange(nph) + 0.5) * (2 * np.pi) / nph
    T, P = np.meshgrid(th, ph, indexing="ij")
    dw = np.sin(T) * (np.pi / 2 / nth) * (2 * np.pi / nph)
    L = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1)
    V = np.array([np.sqrt(max(0.0, 1 - mu * mu)), 0.0, mu])
    fe, pe = disney_eval_nonmetal(np.broadcast_to(V, L.shape), L, roughness, ior, clearcoat, gloss, base)
    fo, _ = disney_eval_nonmetal(np.broadcast_to(V, L.shape), L, roughness, ior, 0.0, gloss, base)
    # fo: the diffuse + specular part of f_eval (clearcoat 0 drops only its f term; its pdf
    # weights are not used here)
    pl = 1.0 / (2 * np.pi ** 2 * np.maximum(np.sin(T), 1e-10))
    wl = pl ** 2 / (pl ** 2 + pe ** 2)
    A = float(np.sum(wl * fe * dw))
    B = float(np.sum((1 - wl) * fo * fe / np.where(pe > 0, pe, 1.0) * dw))
    return A, B


@lru_cache(maxsize=None)
def clearcoat_curve_table(roughness: float, ior: float, clearcoat: float, gloss: float, base: float,
                          n_mu: int = 40, n_psi: int = 72, n: int = 1024):
    """clearcoat_curve_term over a grid of V (cosine mu with N, azimuth psi in the local frame):
    the curve is not rotationally symmetric, so the term depends on psi too."""
    mus = np.linspace(0.02, 1.0, n_mu)
    psis = np.linspace(-np.pi, np.pi, n_psi + 1)
    tab = np.zeros((n_mu, n_psi + 1))
    for i, mu in enumerate(mus):
        st = np.sqrt(max(0.0, 1 - mu * mu))
        for j, ps in enumerate(psis[:-1]):
            tab[i, j] = clearcoat_curve_term(np.array([st * np.cos(ps), st * np.sin(ps), mu]), roughness, ior,
                                             clearcoat, gloss, n, base)
        tab[i, -1] = tab[i, 0]
    return mus, psis, tab


def bilinear(mus, psis, tab, mu, psi):
    i = np.clip(np.searchsorted(mus, mu) - 1, 0, len(mus) - 2)
    j = np.clip(np.searchsorted(psis, psi) - 1, 0, len(psis) - 2)
    u = np.clip((mu - mus[i]) / (mus[i + 1] - mus[i]), 0, 1)
    v = np.clip((psi - psis[j]) / (psis[j + 1] - psis[j]), 0, 1)
    return ((1 - u) * (1 - v) * tab[i, j] + u * (1 - v) * tab[i + 1, j] + (1 - u) * v * tab[i, j + 1]
            + u * v * tab[i + 1, j + 1])


def floor_local_view(dirs):
    """V = -ray in the frame getTangent builds for the floor's normal +y (RT:396-407): helper
    (1, 0, 0), bitangent = normalize(cross(N, helper)) = (0, 0, -1), tangent = cross(N, B) = (-1, 0, 0):
    local V = (-V.x, -V.z, V.y)."""
    V = -dirs
    return np.stack([-V[..., 0], -V[..., 2], V[..., 1]], -1)


# ------------------------------------------------------------------ SCATTER slab (Monte Carlo)
def scatter_slab_mc(origins, dirs, y_top: float, thickness: float, bounds, ior: float, color, density: float,
                    le: float, rng, max_bounce: int = 8, variant: str = ""):
    """An independent Monte-Carlo estimate (numpy's own random numbers, analytic plane
    intersections) of the reference BSDF integrator's process for the smooth glass slab with a
    SCATTER medium of anisotropy 0, one path per (origin, dir) camera ray; returns the paths'
    radiance (N, 3).  The process (RT:1369-1516), beyond the slab rules of `slab_expectation`:
      - on a refraction, scatterDist = min(-log(xi_3) / density, hit.distance) with the SAME xi_3
        that chose refraction (xi_3 >= F), hit.distance the arriving segment (R11, the camera
        segment at the first face); when scatterDist < hit.distance the point moves along the
        arriving ray by scatterDist -- past the glass, possibly past the slab -- history *=
        color * exp(-scatterDist) (no density in the exponent, RT:1445-1446), and the next
        direction is SampleHG(V, 0, ...): uniform on the sphere, with evf = evp = PhaseHG = 1 / 4 pi
        (RT:1448-1451, RT:1470-1473);
      - such a ray that escapes adds history * Le * PhaseHG / hdrPdf(L) with no MIS weight
        (RT:1494), hdrPdf of the constant map = 1 / (2 pi^2 sin theta_L);
      - light samples count from the faces' open sides only (shadow rays into the slab hit the
        other face), their MIS-weighted lobe tails `nee_tail`.
    variant "density_exp": the physical transmittance exp(-density * scatterDist) instead."""
    eta = 1.0 / ior
    f0 = ((1.0 - eta) / (1.0 + eta)) ** 2
    color = np.asarray(color, np.float64)
    y_bot = y_top - thickness
    n = len(dirs)
    d = np.array(dirs, np.float64)
    t = (y_top - origins[:, 1]) / d[:, 1]
    pos = origins + t[:, None] * d
    seg = t - 1e-5
    hist = np.ones((n, 3))
    Lo = np.zeros((n, 3))
    alive = np.ones(n, bool)
    a = A_SMOOTH
    (x0, x1), (z0, z1) = bounds

    def g1(mu):
        return smith_g1(mu, 1.0 - mu * mu, a)

    for _ in range(max_bounce):
        idx = np.nonzero(alive)[0]
        if idx.size == 0:
            break
        dd, pp, sg, hh = d[idx], pos[idx], seg[idx], hist[idx]
        mu = np.abs(dd[:, 1])
        on_top = np.abs(pp[:, 1] - y_top) < np.abs(pp[:, 1] - y_bot)
        # the side the ray came from is open sky: the top face hit from above, the bottom from below
        open_side = (on_top & (dd[:, 1] < 0)) | (~on_top & (dd[:, 1] > 0))
        Lo[idx] += np.where(open_side[:, None], hh * le * nee_tail(mu, eta)[:, None], 0.0)
        F = dielectric_fresnel(mu, eta)
        Fs = f0 + (1.0 - f0) * F
        xi3 = rng.random(idx.size)
        refl = xi3 < F
        # reflection: history *= Fs G1 / F; the ray's y flips
        hh = np.where(refl[:, None], hh * (Fs * g1(mu) / F)[:, None], hh)
        nd = dd.copy()
        nd[refl, 1] = -nd[refl, 1]
        # refraction with eta = 1 / IOR (R10): tangential part scaled by eta, through the face
        tr = ~refl
        sin2 = eta * eta * (1.0 - mu[tr] ** 2)
        nd[tr, 0] *= eta
        nd[tr, 2] *= eta
        nd[tr, 1] = np.sign(dd[tr, 1]) * np.sqrt(1.0 - sin2)
        mu_out = np.abs(nd[:, 1])
        ratio = np.where(refl, g1(mu_out) * (Fs + 1.0 - F), g1(mu_out) * eta * eta * (Fs + 1.0 - F))
        # SCATTER on refraction
        with np.errstate(divide="ignore"):
            sdist = np.minimum(-np.log(xi3) / density, sg)
        med = tr & (sdist < sg)
        k_ext = density if variant == "density_exp" else 1.0
        hh = np.where(med[:, None], hh * color * np.exp(-k_ext * sdist)[:, None], hh)
        pp = np.where(med[:, None], pp + dd * sdist[:, None], pp)
        m = int(med.sum())
        if m:
            cz = 1.0 - 2.0 * rng.random(m)
            ph = 2 * np.pi * rng.random(m)
            sz = np.sqrt(np.maximum(0.0, 1.0 - cz * cz))
            nd[med] = np.stack([sz * np.cos(ph), cz, sz * np.sin(ph)], -1)  # uniform: the axis is moot
        # continuation: nearest face within the quad at t >= 0.0005 (RT:268)
        best = np.full(idx.size, np.inf)
        for y in (y_top, y_bot):
            with np.errstate(divide="ignore", invalid="ignore"):
                tt = (y - pp[:, 1]) / nd[:, 1]
            hx = pp[:, 0] + tt * nd[:, 0]
            hz = pp[:, 2] + tt * nd[:, 2]
            hit = (tt >= 0.0005) & (hx >= x0) & (hx <= x1) & (hz >= z0) & (hz <= z1)
            best = np.where(hit & (tt < best), tt, best)
        esc = ~np.isfinite(best)
        sin_l = np.sqrt(np.maximum(0.0, 1.0 - nd[:, 1] ** 2))
        w_esc = np.where(med, (1.0 / (4 * np.pi)) * 2 * np.pi ** 2 * np.maximum(sin_l, 1e-10), ratio)
        Lo[idx] += np.where(esc[:, None], hh * le * w_esc[:, None], 0.0)
        alive[idx[esc]] = False
        keep = ~esc
        k = idx[keep]
        d[k] = nd[keep]
        pos[k] = pp[keep] + best[keep, None] * nd[keep]
        seg[k] = best[keep] - 1e-5
        hist[k] = hh[keep]
    return Lo
