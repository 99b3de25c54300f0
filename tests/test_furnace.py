"""White-furnace tests: physics the reference's integrator must satisfy, independent of the code.

Every other parity test compares the HIP path with the oracle, and both restate the same GLSL
lines (a slip in both would pass).  These checks do not use the GLSL at all:
inside a uniform environment of radiance Le, a metal with base colour 1 (Schlick F = F0 = 1 for
every angle, RT:397-405) reflects all the light that its microfacet model keeps, so

- every pixel that misses the object equals Le * envIntensity (RT:1530-1536, the env lookup of
  a constant map), whatever the direction;
- with MIS (RT:1380-1405 light sample + RT:1420-1503 BSDF sample weighted by misMixWeight,
  RT:1226-1229) the mean over the object's pixels is Le * envIntensity up to the energy the
  lobe loses.  Near-specular (roughness 0.05 / 0.1) it loses almost nothing: the mean is 1
  within 0.5% / 1%.  A wrong hdrPdf or SampleHdr, a light or BSDF pdf off by a factor, a MIS
  weight that does not sum to one, or a VNDF sample/eval mismatch moves it by far more.
- at any roughness the mean never exceeds 1 (plus sampling error), and the loss grows with
  roughness.  It grows faster than single-scattering GGX alone because the reference applies
  the sampled bounce's weight twice to an escaping path: history *= f/pdf (RT:1431), then
  Lo += history * light * f_eval/pdf_eval of the same direction (RT:1496) -- for F = 1 metal
  that is G1(L)^2 instead of G1(L).  This test found that property of the reference (roughness
  0.6: 0.75, 0.8: 0.50 of the furnace); both implementations keep it (R-faithful).
- the BRDF integrator (enableBSDF off) samples GTR2 half-vectors (RT:1290-1367) and has the
  same double weight (RT:1338 then RT:1352): 1 within 2% at roughness 0.05, monotone after.
  On the plane its non-metal materials are pinned as well: the Disney diffuse lobe (Fd90
  retro-reflection) plus the Schlick specular, sampled as a lobe mixture (RT:789-833).
- the BSDF integrator's non-metals (transmission 0) on the plane: EvalDiffuse + the
  dielectric-Fresnel EvalSpecReflection with DisneyEval's Fresnel-based lobe weights.

The furnace is a constant 64x32 HDR map (its hdrCache from the same host code as the real
map's, `rts_hdr_cache`); the object is the reference's bunny mesh in front of the camera.
The GPU tests also require the HIP image to equal the oracle's bit for bit, and repeat the
furnace at 1920x1080 (a size-independent property, no oracle).

The plane tests go one step further and pin the *value* of the reference's estimator, not just
a bound: for a flat floor of F = 1 metal in the furnace every path ends after one bounce, so the
expected pixel value is a 2-D integral over the hemisphere that numpy evaluates from the BSDF's
formulas alone (GGX D, separable Smith G1 with alpha = roughness^2, RT:447-471; the VNDF pdf
G1(V) D / (4 V.z), RT:962; hdrPdf of a constant map 1 / (2 pi^2 sin theta), RT:1173-1186; the
power-heuristic MIS of RT:1285-1288 on both estimators; the double weight above).  No sampling
routine enters the integral, so SampleGGXVNDF, SampleHdr, the Sobol/Cranley-Patterson numbers
and the wavefront bookkeeping are all checked against it: the mean over the floor's pixels must
equal the integral within 0.2% plus the sampling error (measured on the oracle at 480x270x16
with a 512- or 2048-wide map: 0.05% / 0.14% below it at roughness 0.5 / 0.8, 1-2 standard
errors; a missing double weight or a pdf off by any factor moves it by 10% and more).

Not covered, by the reference's own design: a dielectric (RT:1429 skips f/pdf on refraction,
R9) and the Disney diffuse lobe (retro-reflection, albedo != 1) are not energy conserving, and
with MIS off the light sample and the BSDF sample both count the environment (RT:1396, :1431),
so those cases have no furnace value to test against.
"""
from functools import lru_cache

import numpy as np
import pytest

from helpers import bit_mismatch, frames_for, gpu_render, oracle_render
from rtamd import configs as cf
from rtamd import scene_lib as sl

LE = 0.75            # furnace radiance
INTENSITY = 2.0      # envIntensity (RT:1536): the expected radiance is LE * INTENSITY = 1.5
EXPECT = np.float32(LE) * np.float32(INTENSITY)
# the bunny 3 units along the default camera's front vector, scaled to fill the middle of the frame
BUNNY_AT = ((0, 0, 0), (0.1128, -0.7258, 4.0913), (2.5, 2.5, 2.5))
# roughness -> (lower bound of the object's mean / EXPECT, upper bound), BSDF integrator
BOUNDS = {0.05: (0.995, 1.005), 0.1: (0.99, 1.005), 0.3: (0.0, 1.005), 0.6: (0.0, 1.005)}
# BRDF integrator (enableBSDF off, RT:1290-1367: GTR2 half-vector sampling, not the VNDF)
BOUNDS_BRDF = {0.05: (0.98, 1.005), 0.1: (0.0, 1.005), 0.3: (0.0, 1.005), 0.6: (0.0, 1.005)}
MODES = {"bsdf": (True, BOUNDS), "brdf": (False, BOUNDS_BRDF)}


def furnace_env():
    img = np.full((32, 64, 3), LE, np.float32)
    return img, sl.hdr_cache(img)


def furnace_scene(roughness: float):
    mat = sl.Material(base_color=(1.0, 1.0, 1.0), metallic=1.0, roughness=roughness, specular=1.0)
    return cf.build_scene((cf.Obj("bunny_4000", mat, *BUNNY_AT, False),))


def furnace_stats(img):
    """(fraction of object pixels, their mean / EXPECT, its standard error, max miss error)."""
    v = np.asarray(img, np.float64) / float(EXPECT)
    miss = np.all(np.abs(v - 1.0) < 1e-6, axis=-1)
    obj = v[~miss].mean(axis=-1)
    return float((~miss).mean()), float(obj.mean()), float(obj.std() / np.sqrt(max(obj.size, 1)))


def check_furnace(img, roughness, bounds=BOUNDS):
    frac, mean, se = furnace_stats(img)
    lo, hi = bounds[roughness]
    assert 0.1 < frac < 0.9, f"object covers {frac:.2f} of the frame"
    assert np.isfinite(img).all()
    assert lo - 4 * se <= mean <= hi + 4 * se, f"roughness {roughness}: mean {mean:.4f} +- {se:.4f}"
    return mean


def test_constant_env_cache_is_uniform():
    """calculateHdrCache (Scene.h:165-215) of a constant map: every texel has the same pdf,
    1 / texel count (hdrPdf divides by the sphere's 2*pi^2*sin(theta) Jacobian later)."""
    img, cache = furnace_env()
    assert np.isfinite(cache).all()
    assert np.all(cache[..., 2] == np.float32(1.0 / (64 * 32)))


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("roughness", sorted(BOUNDS))
def test_oracle_white_furnace(roughness, mode):
    bsdf, bounds = MODES[mode]
    W, H = 64, 36
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=bsdf)
    _, frames = frames_for(fp, 1, 32)
    img, cnt = oracle_render(furnace_scene(roughness), furnace_env(), W, H, frames)
    assert cnt["rays"] > 0
    check_furnace(img, roughness, bounds)


@pytest.mark.parametrize("mode", list(MODES))
def test_oracle_furnace_loss_grows_with_roughness(mode):
    W, H = 64, 36
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=MODES[mode][0])
    _, frames = frames_for(fp, 1, 32)
    means = [furnace_stats(oracle_render(furnace_scene(r), furnace_env(), W, H, frames)[0])[1]
             for r in sorted(BOUNDS)]
    assert all(a > b for a, b in zip(means, means[1:])), means


@pytest.mark.gpu
@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("roughness", sorted(BOUNDS))
def test_gpu_white_furnace_matches_oracle(gpu_renderer, roughness, mode):
    bsdf, bounds = MODES[mode]
    sd, env = furnace_scene(roughness), furnace_env()
    W, H = 64, 36
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=bsdf)
    ro, frames = frames_for(fp, 1, 32)
    ref, cnt = oracle_render(sd, env, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env, W, H, fp, ro)
    assert st["rays"] == cnt["rays"]
    frac, diff = bit_mismatch(img, ref)
    assert frac == 0.0, f"{int(diff.sum())} of {W * H} pixels differ"
    check_furnace(img, roughness, bounds)


@pytest.mark.gpu
@pytest.mark.parametrize("roughness", [0.05, 0.6])
def test_gpu_white_furnace_full_hd(gpu_renderer, roughness):
    """The furnace at the configurations' size, 16 frames: a property check, no oracle."""
    sd, env = furnace_scene(roughness), furnace_env()
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    ro, _ = frames_for(fp, 1, 16)
    img, st = gpu_render(gpu_renderer, sd, env, W, H, fp, ro)
    assert st["rays"] >= W * H * 16
    check_furnace(img, roughness)


# ------------------------------------------------------------------ plane: the estimator's value
FLOOR_AT = ((0, 0, 0), (2.2, -2, 3), (14, 7, 7))   # the reference's floor (Scene.h:116-120): y = const


def estimator_terms(mu: float, roughness: float, nth: int = 200, nph: int = 400, brdf: bool = False,
                    metallic: float = 1.0, specular: float = 1.0, ior: float = 1.5,
                    clearcoat: float = 0.0, gloss: float = 0.5, sheen: float = 0.0):
    """The reference BSDF integrator's expectation for one bounce off an F = 1 metal plane
    (normal = +y = the env map's pole axis) viewed at cosine mu, as three hemisphere integrals
    (midpoint rule): A = the light sample, w_l f cos (RT:1380-1405, the constant-map hdrPdf
    cancels); B = the escaping BSDF sample with its MIS weight, p_b w_b (f cos / p_b)^2 (RT:1431,
    RT:1496); S[c] = the same sample in sky mode, p_b (f cos / p_b)^2 getDefaultSkyColor(L.y)[c]
    (RT:1500-1503: no MIS weight, no envIntensity; RT:1190-1193).
    brdf: the BRDF integrator instead (RT:1290-1367, the same three terms at RT:1321, :1338 + :1352,
    :1356) with BRDF_Evaluate's metal specular (RT:836-920): GTR2(NdotH, roughness^2), Smith G1
    with alphaG = roughness (RT:876-877, not roughness^2) and the GTR2 half-vector pdf
    D NdotH / (4 LdotH) of SampleGTR2 (RT:732-749, :911)."""
    a = max(1e-3, roughness * roughness)                       # m.ax = m.ay (RT:205-207)
    th = (np.arange(nth) + 0.5) * (np.pi / 2) / nth
    ph = (np.arange(nph) + 0.5) * (2 * np.pi) / nph
    T, P = np.meshgrid(th, ph, indexing="ij")
    dw = np.sin(T) * (np.pi / 2 / nth) * (2 * np.pi / nph)
    L = np.stack([np.sin(T) * np.cos(P), np.sin(T) * np.sin(P), np.cos(T)], -1)
    V = np.array([np.sqrt(max(0.0, 1 - mu * mu)), 0.0, mu])
    Hh = L + V
    Hh /= np.linalg.norm(Hh, axis=-1, keepdims=True)
    D = 1.0 / (np.pi * a * a * ((Hh[..., 0] / a) ** 2 + (Hh[..., 1] / a) ** 2 + Hh[..., 2] ** 2) ** 2)

    def G1(w):
        return 2 * w[..., 2] / (w[..., 2] + np.sqrt(a * a * (w[..., 0] ** 2 + w[..., 1] ** 2) + w[..., 2] ** 2))

    if brdf:
        def G1(w):  # SmithG_GGX(NdotV, alphaG = roughness): a = roughness^2 under the root
            r2 = roughness * roughness
            return 2 * w[..., 2] / (w[..., 2] + np.sqrt(r2 + w[..., 2] ** 2 - r2 * w[..., 2] ** 2))

    def G1b025(w):  # SmithG_GGX(NdotV, 0.25) of the clearcoat (RT:892)
        return 2 * w[..., 2] / (w[..., 2] + np.sqrt(0.0625 + w[..., 2] ** 2 - 0.0625 * w[..., 2] ** 2))

    g1v, g1l = G1(V), G1(L)
    fcos = D * g1v * g1l / (4 * mu)       # F D G2 / (4 L.z V.z) * L.z, F = 1
    p_true = None                         # the sampling density, when it is not the eval's pdf
    if brdf:
        LdotH = np.sum(L * Hh, axis=-1)
        pb = D * Hh[..., 2] / (4 * LdotH)   # GTR2 half-vector pdf
        if metallic < 1.0:
            # BRDF_Evaluate with base colour 1 (Ctint = 1): Disney diffuse Fd / pi, specular with
            # Fs = mix(Cspec0, 1, FH), Cspec0 = mix(0.08 * specular, 1, metallic); lobe choice
            # p_diffuse : p_specular = (1 - metallic) : 1 (CalculateBRDFLobePdfs, RT:520-533)
            def schlick(u):
                return np.clip(1.0 - u, 0.0, 1.0) ** 5
            fd90 = 0.5 + 2.0 * LdotH * LdotH * roughness
            Fd = (1 + (fd90 - 1) * schlick(L[..., 2])) * (1 + (fd90 - 1) * schlick(mu))
            cspec0 = 0.08 * specular * (1 - metallic) + metallic
            Fs = cspec0 + (1 - cspec0) * schlick(LdotH)
            # sheen (RT:894, :898): FH * sheen * Csheen added to the diffuse term, Csheen = 1 here
            fcos = ((1 - metallic) * (Fd / np.pi + schlick(LdotH) * sheen)) * L[..., 2] + Fs * fcos
            rc = (1 - metallic) * 0.25 * clearcoat
            rsum = (1 - metallic) + 1 + rc
            pd, ps, pc = (1 - metallic) / rsum, 1 / rsum, rc / rsum
            ps_spec = pb
            pb = pd * L[..., 2] / np.pi + ps * pb
            if clearcoat > 0:
                # clearcoat (RT:890-900): GTR1 with alpha mix(0.1, 0.001, 1 - gloss) in the eval
                # but mix(0.1, 0.001, gloss) in SampleGTR1 (RT:797, :825): the eval's pdf is not
                # the sampling density unless gloss = 0.5, and the BRDF integrator divides by the
                # eval's pdf (RT:1338), so the density enters the expectation (returned as ps_true)
                def gtr1(c, al):
                    a2 = al * al
                    return (a2 - 1) / (np.pi * np.log(a2) * (1 + (a2 - 1) * c * c))
                ae, as_ = 0.1 + (0.001 - 0.1) * (1 - gloss), 0.1 + (0.001 - 0.1) * gloss
                Dr = gtr1(Hh[..., 2], ae)
                Fr = 0.04 + 0.96 * schlick(LdotH)
                Gr = G1b025(L) * G1b025(V)
                fcos = fcos + 0.25 * Gr * Fr * Dr * clearcoat / (4 * mu)
                pb = pb + pc * Dr * Hh[..., 2] / (4 * LdotH)
                p_true = (pd * L[..., 2] / np.pi + ps * ps_spec
                          + pc * gtr1(Hh[..., 2], as_) * Hh[..., 2] / (4 * LdotH))
    else:
        pb = g1v * D / (4 * mu)           # VNDF pdf of the reflected direction
        if metallic < 1.0:
            # DisneyEval of a non-metal, transmission 0, base colour 1 (RT:1010-1067): EvalDiffuse
            # (Fd90) + EvalSpecReflection with F = mix(specCol, 1, DielectricFresnel(V.H, eta)),
            # specCol = F0^2 (GetSpecColor, RT:420-427), lobe weights from that same Fresnel
            # (CalculateBSDFLobePdfs, RT:537-550).  The sample's own pdf (approxFresnel weights)
            # cancels: history carries f_lobe / p_lobe, the escape multiplies by f / p_eval.
            eta = 1.0 / ior
            LdotH = np.sum(L * Hh, axis=-1)
            VdotH = np.abs(np.sum(V * Hh, axis=-1))
            sin2 = eta * eta * (1 - VdotH * VdotH)
            cost = np.sqrt(np.maximum(1 - sin2, 0.0))
            rs = (eta * cost - VdotH) / (eta * cost + VdotH)
            rp = (eta * VdotH - cost) / (eta * VdotH + cost)
            fres = 0.5 * (rs * rs + rp * rp)
            F0 = ((1 - eta) / (1 + eta)) ** 2
            Fspec = F0 + (1 - F0) * fres

            def schlick(u):
                return np.clip(1.0 - u, 0.0, 1.0) ** 5
            fd90 = 0.5 + 2.0 * LdotH * LdotH * roughness
            Fd = (1 + (fd90 - 1) * schlick(L[..., 2])) * (1 + (fd90 - 1) * schlick(mu))
            wd = 1.0 / (1.0 + Fspec)
            # EvalDiffuse's sheen (RT:943-946): FH * sheen * sheenCol, sheenCol = 1 here
            fcos = (Fd / np.pi + schlick(LdotH) * sheen) * L[..., 2] + Fspec * fcos
            pb = wd * L[..., 2] / np.pi + (1 - wd) * pb
    pl = 1.0 / (2 * np.pi ** 2 * np.maximum(np.sin(T), 1e-10))
    wl = pl ** 2 / (pl ** 2 + pb ** 2)
    t = 0.5 * (np.cos(T) + 1.0)
    sky = [(1 - t) + t * c for c in (0.5, 0.7, 1.0)]
    A = float(np.sum(wl * fcos * dw))
    # p_s (f cos / p_b)^2: the sample's weight applied twice (p_s = p_b unless p_true says otherwise)
    w2 = fcos * fcos / pb if p_true is None else p_true * (fcos / pb) ** 2
    B = float(np.sum((1 - wl) * w2 * dw))
    S = np.array([np.sum(w2 * sc * dw) for sc in sky])
    return A, B, S


MU_GRID = np.linspace(0.02, 1.0, 80)


@lru_cache(maxsize=None)
def terms_table(roughness: float, brdf: bool = False, metallic: float = 1.0, specular: float = 1.0,
                ior: float = 1.5, clearcoat: float = 0.0, gloss: float = 0.5, sheen: float = 0.0):
    """estimator_terms over MU_GRID (the tests interpolate per pixel between these)."""
    return [estimator_terms(float(m), roughness, brdf=brdf, metallic=metallic, specular=specular, ior=ior,
                            clearcoat=clearcoat, gloss=gloss, sheen=sheen) for m in MU_GRID]


def estimator_expectation(mu: float, roughness: float, brdf: bool = False) -> float:
    """Environment mode, relative to Le * envIntensity: A + B."""
    A, B, _ = estimator_terms(mu, roughness, brdf=brdf)
    return A + B


def view_cosines(fp, W, H):
    """cos(angle between the floor normal +y and -ray) of every pixel's camera ray (RT:1520-1527),
    rows bottom-up as the accumulation buffer stores them."""
    lbc, right, up = (np.asarray(x, np.float64) for x in (fp.left_bottom_corner, fp.right, fp.up))
    u = (np.arange(W) + 0.5) / W
    v = (np.arange(H) + 0.5) / H
    d = (lbc[None, None, :] + (u[None, :, None] * 2 * fp.half_w) * right[None, None, :]
         + (v[:, None, None] * 2 * fp.half_h) * up[None, None, :])
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    return -d[..., 1]


def check_plane(img, fp, W, H, roughness, rel_tol, brdf=False, metallic=1.0, specular=1.0, ior=1.5,
                clearcoat=0.0, gloss=0.5, sheen=0.0):
    v = np.asarray(img, np.float64).mean(axis=-1) / float(EXPECT)
    mu = view_cosines(fp, W, H)
    on = (np.abs(v - 1.0) > 1e-6) & (mu > 0.02)
    assert on.sum() > 0.2 * W * H, on.sum()
    e = np.interp(mu[on], MU_GRID, [A + B for A, B, _ in terms_table(roughness, brdf, metallic, specular, ior, clearcoat, gloss, sheen)])
    got, want = v[on].mean(), e.mean()
    se = v[on].std() / np.sqrt(on.sum())
    assert abs(got - want) <= rel_tol * want + 4 * se, f"roughness {roughness}: {got:.5f} vs {want:.5f} +- {se:.5f}"
    return got / want


@lru_cache(maxsize=1)
def plane_env():
    """A constant 1024x512 map: SampleHdr returns texel-centre directions, so the light sample is
    a quadrature over the map's texels; at 64x32 that quadrature is 0.2-0.4% off the integral,
    at 512 and above it has converged (0.05% / 0.14% below it at roughness 0.5 / 0.8)."""
    img = np.full((512, 1024, 3), LE, np.float32)
    return img, sl.hdr_cache(img)


def floor_scene(roughness: float, metallic: float = 1.0, specular: float = 1.0, ior: float = 1.5,
                clearcoat: float = 0.0, gloss: float = 0.0, sheen: float = 0.0):
    mat = sl.Material(base_color=(1.0, 1.0, 1.0), metallic=metallic, roughness=roughness, specular=specular,
                      ior=ior, clearcoat=clearcoat, clearcoat_gloss=gloss, sheen=sheen)
    return cf.build_scene((cf.Obj("floor", mat, *FLOOR_AT, False),))


@pytest.mark.parametrize("mode", ["bsdf", "brdf"])
@pytest.mark.parametrize("roughness", [0.5, 0.8])
def test_oracle_plane_furnace_equals_estimator_integral(roughness, mode):
    W, H = 48, 27
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=(mode == "bsdf"))
    _, frames = frames_for(fp, 1, 64)
    img, _ = oracle_render(floor_scene(roughness), plane_env(), W, H, frames)
    check_plane(img, fp, W, H, roughness, rel_tol=0.002, brdf=(mode == "brdf"))


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["bsdf", "brdf"])
@pytest.mark.parametrize("roughness", [0.5, 0.8])
def test_gpu_plane_furnace_full_hd_equals_estimator_integral(gpu_renderer, roughness, mode):
    """1920x1080, 8 frames on the GPU against the integral (no oracle): sampling error ~1e-4."""
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=(mode == "bsdf"))
    ro, _ = frames_for(fp, 1, 8)
    img, _ = gpu_render(gpu_renderer, floor_scene(roughness), plane_env(), W, H, fp, ro)
    check_plane(img, fp, W, H, roughness, rel_tol=0.002, brdf=(mode == "brdf"))


def test_oracle_plane_furnace_sky_mode_equals_estimator_integral():
    """Sky mode (enableEnvMap off): the light sample still comes from the HDR map (RT:1379-1405 has
    no enableEnvMap test), the escaping BSDF sample sees getDefaultSkyColor unweighted."""
    W, H, rough = 48, 27, 0.5
    fp_env = cf.frame_params(W, H, env_intensity=INTENSITY)
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_env_map=False)
    _, fr_env = frames_for(fp_env, 1, 1)
    _, frames = frames_for(fp, 1, 64)
    sd = floor_scene(rough)
    env_img, _ = oracle_render(sd, plane_env(), W, H, fr_env)
    img, _ = oracle_render(sd, plane_env(), W, H, frames)
    mu = view_cosines(fp, W, H)
    on = (np.abs(np.asarray(env_img, np.float64).mean(-1) / float(EXPECT) - 1.0) > 1e-6) & (mu > 0.02)
    assert on.sum() > 0.2 * W * H
    for c in range(3):
        tab = [float(EXPECT) * A + S[c] for A, _, S in terms_table(rough)]
        e = np.interp(mu[on], MU_GRID, tab)
        got = np.asarray(img, np.float64)[..., c][on]
        se = got.std() / np.sqrt(on.sum())
        assert abs(got.mean() - e.mean()) <= 0.002 * e.mean() + 4 * se, (c, got.mean(), e.mean(), se)


# BRDF integrator, non-metals: Disney diffuse (Fd90 retro-reflection) + Schlick specular, lobes
# picked 1 : 1 (metallic 0) or 1 : 2 (metallic 0.5); (metallic, specular)
BRDF_MATS = {"plastic": (0.0, 0.5), "diffuse_only_f0": (0.0, 0.0), "half_metal": (0.5, 0.5)}


@pytest.mark.parametrize("mat", list(BRDF_MATS))
@pytest.mark.parametrize("roughness", [0.5, 0.8])
def test_oracle_plane_furnace_brdf_diffuse_equals_estimator_integral(roughness, mat):
    met, spec = BRDF_MATS[mat]
    W, H = 48, 27
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=False)
    _, frames = frames_for(fp, 1, 64)
    img, _ = oracle_render(floor_scene(roughness, met, spec), plane_env(), W, H, frames)
    check_plane(img, fp, W, H, roughness, rel_tol=0.002, brdf=True, metallic=met, specular=spec)


@pytest.mark.gpu
@pytest.mark.parametrize("mat", ["plastic", "half_metal"])
def test_gpu_plane_furnace_brdf_diffuse_full_hd(gpu_renderer, mat):
    met, spec = BRDF_MATS[mat]
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=False)
    ro, _ = frames_for(fp, 1, 8)
    img, _ = gpu_render(gpu_renderer, floor_scene(0.5, met, spec), plane_env(), W, H, fp, ro)
    check_plane(img, fp, W, H, 0.5, rel_tol=0.002, brdf=True, metallic=met, specular=spec)


@pytest.mark.parametrize("ior", [1.5, 1.2])
@pytest.mark.parametrize("roughness", [0.3, 0.8])
def test_oracle_plane_furnace_bsdf_dielectric_equals_estimator_integral(roughness, ior):
    """BSDF integrator, non-metal (transmission 0): Disney diffuse + dielectric-Fresnel specular,
    the eval's lobe weights from that Fresnel, the sample's approxFresnel weights cancelling."""
    W, H = 48, 27
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    _, frames = frames_for(fp, 1, 64)
    img, _ = oracle_render(floor_scene(roughness, 0.0, 0.5, ior), plane_env(), W, H, frames)
    check_plane(img, fp, W, H, roughness, rel_tol=0.002, metallic=0.0, ior=ior)


@pytest.mark.gpu
def test_gpu_plane_furnace_bsdf_dielectric_full_hd(gpu_renderer):
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    ro, _ = frames_for(fp, 1, 8)
    img, _ = gpu_render(gpu_renderer, floor_scene(0.5, 0.0, 0.5, 1.5), plane_env(), W, H, fp, ro)
    check_plane(img, fp, W, H, 0.5, rel_tol=0.002, metallic=0.0, ior=1.5)


@pytest.mark.parametrize("gloss", [0.1, 0.5, 0.9])
def test_oracle_plane_furnace_brdf_clearcoat_equals_estimator_integral(gloss):
    """BRDF integrator with clearcoat 1 (RT:890-900): GTR1 evaluated with alpha
    mix(0.1, 0.001, 1 - gloss) but sampled with mix(0.1, 0.001, gloss) (RT:797, :825); the
    integral uses the sampling density where the estimator divides by the eval's pdf."""
    W, H = 48, 27
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=False)
    _, frames = frames_for(fp, 1, 256)  # a lobe worth 2-5%: a tighter sampling error
    img, _ = oracle_render(floor_scene(0.5, 0.0, 0.5, 1.5, 1.0, gloss), plane_env(), W, H, frames)
    check_plane(img, fp, W, H, 0.5, rel_tol=0.002, brdf=True, metallic=0.0, specular=0.5, clearcoat=1.0, gloss=gloss)


@pytest.mark.parametrize("sheen", [0.5, 1.0])
def test_oracle_plane_furnace_brdf_sheen_equals_estimator_integral(sheen):
    """BRDF integrator with sheen (RT:894, :898): FH * sheen * Csheen joins the diffuse term
    without the 1/pi, sampled by the diffuse lobe."""
    W, H = 48, 27
    fp = cf.frame_params(W, H, env_intensity=INTENSITY, enable_bsdf=False)
    _, frames = frames_for(fp, 1, 256)  # a lobe worth 2-5%: a tighter sampling error
    img, _ = oracle_render(floor_scene(0.5, 0.0, 0.5, sheen=sheen), plane_env(), W, H, frames)
    check_plane(img, fp, W, H, 0.5, rel_tol=0.002, brdf=True, metallic=0.0, specular=0.5, sheen=sheen)


def test_oracle_plane_furnace_bsdf_sheen_equals_estimator_integral():
    """BSDF integrator, EvalDiffuse's sheen term (RT:943-946), sampled by the diffuse lobe."""
    W, H = 48, 27
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    _, frames = frames_for(fp, 1, 256)
    img, _ = oracle_render(floor_scene(0.5, 0.0, 0.5, 1.5, sheen=1.0), plane_env(), W, H, frames)
    check_plane(img, fp, W, H, 0.5, rel_tol=0.002, metallic=0.0, ior=1.5, sheen=1.0)
