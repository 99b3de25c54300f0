"""Furnace pins of the branches the plane furnace (tests/test_furnace.py) does not reach: the
expected pixel comes from tests/furnace_models.py, a numpy evaluation of the GLSL's formulas with
no sampling routine of either implementation in it, and the oracle (small frames) and the GPU
(1920x1080, no oracle) must both equal it.

* Glass slab, roughness 0 (two copies of the reference's floor quad 0.25 apart, IOR 1.5, constant
  1024x512 environment): every path is a chain of reflect / refract choices at the two faces.
  - no medium: pins R9 (a refraction skips f / pdf; the escaping ray's eval weight is G1 eta^2
    (Fs + 1 - F)) and R10 (eta = 1 / IOR leaving the glass too);
  - ABSORB: exp(-(1 - color) density hit.distance) where hit.distance is the segment that arrived
    at the refracting face -- for the first face the camera-to-glass distance (R11);
  - EMISSIVE: Lo += color hit.distance density history at every refraction (RT:1437-1439), the
    camera segment included;
  - SCATTER (anisotropy 0): the free-flight distance min(-log(xi_3) / density, hit.distance) with
    the xi_3 that chose refraction, the point moved along the arriving ray (past the glass, and past
    the slab when the camera segment is long), history *= color exp(-distance) with no density in
    the exponent, a uniform new direction, and an escape weighted by PhaseHG / hdrPdf without MIS
    (RT:1440-1457, RT:1494).  The expectation is a random walk through the slab, so here the
    model is an independent Monte-Carlo estimate (numpy's generator, analytic plane hits,
    `furnace_models.scatter_slab_mc`) and its own standard error joins the tolerance.
  The model tells these behaviours apart from their physical readings by 10-50x the tolerance
  (`test_slab_model_tells_the_quirks_apart`).
* BSDF integrator clearcoat alone (base colour 0, IOR 1: the diffuse and specular lobes weigh 0):
  EvalClearcoat's GTR1 with alpha = clearcoatGloss (R23, RT:994), its Fresnel / Smith terms and
  lobe pdf, the MIS weights, and SampleGTR1(rgh, r1, r2) drawing theta AND phi from r1 (R23,
  RT:716-729) as a 1-D integral.  (That sampler's curve and a proper 2-D draw give expectations
  within ~0.2% of each other on this floor -- the integrand is nearly symmetric about N -- so
  the sampler's r1 reuse itself is only weakly separated; the eval's alpha is strongly.)

Tolerance: 0.2% of the expected mean plus 4 standard errors of the image mean.  NaN pixels are
the reference's own R14 (a CP-rotated Sobol value of exactly 1.0 gives a grazing VNDF normal whose
refraction has eval pdf 0, so Le * f / 0 = NaN: 1 in ~10^7 paths); they are excluded and counted.
"""
from functools import lru_cache

import numpy as np
import pytest

import furnace_models as fm
from helpers import frames_for, gpu_render, oracle_render
from rtamd import configs as cf
from rtamd import scene_lib as sl
from test_furnace import EXPECT, FLOOR_AT, INTENSITY, plane_env

SLAB_H = 0.25
SLAB_TOP = -2.0      # the floor quad's plane (Scene.h:116-120)
MEDIA = {  # name -> (medium type, colour, density)
    "none": (0, (1.0, 1.0, 1.0), 0.0),
    "absorb": (1, (0.9, 0.6, 0.3), 0.08),
    "emissive": (3, (0.2, 0.5, 0.9), 0.5),
    "scatter": (2, (0.8, 0.5, 0.2), 0.15),
}
REL_TOL = 0.002


def slab_scene(medium: str):
    mt, col, dens = MEDIA[medium]
    mat = sl.Material(base_color=(1.0, 1.0, 1.0), transmission=1.0, ior=1.5, roughness=0.0, specular=1.0,
                      medium_type=mt, medium_color=col, medium_density=dens)
    r, t, s = FLOOR_AT
    return cf.build_scene((cf.Obj("floor", mat, r, t, s, False),
                           cf.Obj("floor", mat, r, (t[0], t[1] - SLAB_H, t[2]), s, False)))


def slab_expected(sd, fp, W, H, medium: str, variant: str = ""):
    """(expected image, mask of the pixels whose every path stays inside the quads)"""
    _, col, dens = MEDIA[medium]
    dirs = fm.camera_rays(fp, W, H)
    cam = np.asarray(cf.CAMERA_POSITION, np.float64)
    exp, travel = fm.slab_expectation(dirs, cam, SLAB_TOP, SLAB_H, 1.5, {0: "none", 1: "absorb", 3: "emissive"}[
        MEDIA[medium][0]], col, dens, float(EXPECT), variant=variant)
    p = np.concatenate([sd.soa[k].reshape(-1, 3) for k in ("p1", "p2", "p3")])
    lo, hi = p.min(0), p.max(0)
    t0 = (SLAB_TOP - cam[1]) / dirs[..., 1]
    P0 = cam + t0[..., None] * dirs
    m = travel + 0.2
    ok = ((dirs[..., 1] < 0) & (P0[..., 0] > lo[0] + m) & (P0[..., 0] < hi[0] - m) & (P0[..., 2] > lo[2] + m)
          & (P0[..., 2] < hi[2] - m))
    return exp, ok


def check_mean(img, exp, ok, what, max_nan=0.0005, want_mean=None, want_se=None):
    """Per channel: the image's mean over the `ok` pixels equals the model's (the per-pixel
    expectation `exp`, or a Monte-Carlo mean `want_mean` with its standard error `want_se`)
    within REL_TOL plus 4 combined standard errors."""
    img = np.asarray(img, np.float64)
    finite = np.isfinite(img).all(-1)
    assert ok.sum() > 0.03 * ok.size, ok.sum()
    assert (ok & ~finite).sum() <= max(2, max_nan * ok.sum()), (ok & ~finite).sum()
    sel = ok & finite
    for c in range(3):
        got = img[..., c][sel]
        want = exp[..., c][sel].mean() if want_mean is None else want_mean[c]
        se = np.hypot(got.std() / np.sqrt(got.size), 0.0 if want_se is None else want_se[c])
        assert abs(got.mean() - want) <= REL_TOL * want + 4 * se, \
            f"{what} channel {c}: {got.mean():.5f} vs {want:.5f} +- {se:.5f}"


@pytest.mark.parametrize("medium", ["none", "absorb", "emissive"])
def test_oracle_slab_furnace_equals_model(medium):
    sd = slab_scene(medium)
    W, H = 128, 72
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    _, frames = frames_for(fp, 1, 256)
    img, _ = oracle_render(sd, plane_env(), W, H, frames)
    exp, ok = slab_expected(sd, fp, W, H, medium)
    check_mean(img, exp, ok, medium)


@pytest.mark.parametrize("medium,variant", [("absorb", "r11_physical"), ("emissive", "r11_physical"),
                                            ("none", "r9_weighted"), ("absorb", "r9_weighted")])
def test_slab_model_tells_the_quirks_apart(medium, variant):
    """The physical readings of R11 (the medium acts only inside the glass) and R9 (refraction
    weighted by f / pdf like reflection) move the slab's mean by at least 10x the tolerance."""
    sd = slab_scene(medium)
    W, H = 128, 72
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    exp, ok = slab_expected(sd, fp, W, H, medium)
    alt, _ = slab_expected(sd, fp, W, H, medium, variant)
    rel = np.abs(alt[ok].mean(0) - exp[ok].mean(0)) / exp[ok].mean(0)
    assert rel.max() > 10 * REL_TOL, rel


@pytest.mark.gpu
@pytest.mark.parametrize("medium", ["none", "absorb", "emissive"])
def test_gpu_slab_furnace_full_hd_equals_model(gpu_renderer, medium):
    sd = slab_scene(medium)
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    ro, _ = frames_for(fp, 1, 8)
    img, _ = gpu_render(gpu_renderer, sd, plane_env(), W, H, fp, ro)
    exp, ok = slab_expected(sd, fp, W, H, medium)
    check_mean(img, exp, ok, medium)


def scatter_expected(sd, fp, W, H, n_paths: int, seed: int = 7, variant: str = ""):
    """(pixels whose camera ray hits the top face, Monte-Carlo mean and its standard error per
    channel) of the SCATTER slab, camera rays drawn uniformly over those pixels."""
    _, col, dens = MEDIA["scatter"]
    dirs = fm.camera_rays(fp, W, H)
    cam = np.asarray(cf.CAMERA_POSITION, np.float64)
    p = np.concatenate([sd.soa[k].reshape(-1, 3) for k in ("p1", "p2", "p3")])
    lo, hi = p.min(0), p.max(0)
    t0 = (SLAB_TOP - cam[1]) / dirs[..., 1]
    P0 = cam + t0[..., None] * dirs
    ok = (dirs[..., 1] < 0) & (P0[..., 0] > lo[0]) & (P0[..., 0] < hi[0]) & (P0[..., 2] > lo[2]) & (P0[..., 2] < hi[2])
    rng = np.random.default_rng(seed)
    D = dirs[ok][rng.integers(0, int(ok.sum()), n_paths)]
    Lo = fm.scatter_slab_mc(np.broadcast_to(cam, D.shape), D, SLAB_TOP, SLAB_H, ((lo[0], hi[0]), (lo[2], hi[2])),
                            1.5, col, dens, float(EXPECT), rng, variant=variant)
    return ok, Lo.mean(0), Lo.std(0) / np.sqrt(n_paths)


def test_oracle_scatter_slab_equals_monte_carlo():
    sd = slab_scene("scatter")
    W, H = 128, 72
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    _, frames = frames_for(fp, 1, 512)
    img, _ = oracle_render(sd, plane_env(), W, H, frames)
    ok, m, se = scatter_expected(sd, fp, W, H, 3_000_000)
    check_mean(img, img, ok, "scatter", want_mean=m, want_se=se)


def test_scatter_model_tells_density_in_the_exponent_apart():
    """exp(-scatterDist) (RT:1445) against the physical exp(-density * scatterDist), on the same
    camera rays and random numbers: the mean moves by far more than the tolerance."""
    sd = slab_scene("scatter")
    W, H = 128, 72
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    _, m, se = scatter_expected(sd, fp, W, H, 300_000)
    _, alt, _ = scatter_expected(sd, fp, W, H, 300_000, variant="density_exp")
    assert np.all(np.abs(alt - m) > 10 * REL_TOL * m + 4 * se), (m, alt)


# ------------------------------------------------------------------ clearcoat alone (R23)
def clearcoat_scene(gloss: float):
    mat = sl.Material(base_color=(0.0, 0.0, 0.0), metallic=0.0, roughness=0.5, ior=1.0, clearcoat=1.0,
                      clearcoat_gloss=gloss)
    return cf.build_scene((cf.Obj("floor", mat, *FLOOR_AT, False),))


@lru_cache(maxsize=None)
def _light_table(gloss: float):
    mus = np.linspace(0.02, 1.0, 40)
    with np.errstate(invalid="ignore", divide="ignore"):
        return mus, np.array([sum(fm.bsdf_clearcoat_other_terms(m, 0.5, 1.0, 1.0, gloss, base=0.0)) for m in mus])


def clearcoat_expected(fp, W, H, gloss: float):
    """Per pixel, relative to Le * envIntensity: the light sample A(mu) (isotropic) + the
    clearcoat curve term (mu, azimuth table)."""
    Vl = fm.floor_local_view(fm.camera_rays(fp, W, H))
    mu = Vl[..., 2]
    psi = np.arctan2(Vl[..., 1], Vl[..., 0])
    mus, tab = _light_table(gloss)
    with np.errstate(invalid="ignore", divide="ignore"):
        cm, cp, ct = fm.clearcoat_curve_table(0.5, 1.0, 1.0, gloss, 0.0)
    return np.interp(mu, mus, tab) + fm.bilinear(cm, cp, ct, mu, psi), mu


def check_clearcoat(img, fp, W, H, gloss):
    v = np.asarray(img, np.float64).mean(-1) / float(EXPECT)
    exp, mu = clearcoat_expected(fp, W, H, gloss)
    finite = np.isfinite(v)
    on = (np.abs(v - 1.0) > 1e-6) & (mu > 0.02) & finite
    assert on.sum() > 0.2 * W * H, on.sum()
    assert (~finite).sum() <= max(2, 0.0005 * on.sum())
    got, want = v[on].mean(), exp[on].mean()
    se = v[on].std() / np.sqrt(on.sum())
    assert abs(got - want) <= REL_TOL * want + 4 * se, f"gloss {gloss}: {got:.6f} vs {want:.6f} +- {se:.6f}"


@pytest.mark.parametrize("gloss", [0.1, 0.5, 0.9])
def test_oracle_bsdf_clearcoat_equals_model(gloss):
    W, H = 96, 54
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    _, frames = frames_for(fp, 1, 256)
    img, _ = oracle_render(clearcoat_scene(gloss), plane_env(), W, H, frames)
    check_clearcoat(img, fp, W, H, gloss)


def test_clearcoat_model_tells_eval_alpha_apart():
    """Disney's own GTR1 alpha, mix(0.1, 0.001, gloss) (the comment at RT:994), instead of the
    reference's alpha = gloss moves the expectation far beyond the tolerance."""
    mu = 0.4
    with np.errstate(invalid="ignore", divide="ignore"):
        ref = sum(fm.bsdf_clearcoat_other_terms(mu, 0.5, 1.0, 1.0, 0.5, base=0.0))
        alt = sum(fm.bsdf_clearcoat_other_terms(mu, 0.5, 1.0, 1.0, 0.1 + (0.001 - 0.1) * 0.5, base=0.0))
    assert abs(alt - ref) / ref > 10 * REL_TOL, (ref, alt)


@pytest.mark.gpu
def test_gpu_scatter_slab_full_hd_equals_monte_carlo(gpu_renderer):
    sd = slab_scene("scatter")
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    ro, _ = frames_for(fp, 1, 8)
    img, _ = gpu_render(gpu_renderer, sd, plane_env(), W, H, fp, ro)
    ok, m, se = scatter_expected(sd, fp, W, H, 3_000_000)
    check_mean(img, img, ok, "scatter", want_mean=m, want_se=se)


@pytest.mark.gpu
@pytest.mark.parametrize("gloss", [0.1, 0.9])
def test_gpu_bsdf_clearcoat_full_hd_equals_model(gpu_renderer, gloss):
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, env_intensity=INTENSITY)
    ro, _ = frames_for(fp, 1, 16)
    img, _ = gpu_render(gpu_renderer, clearcoat_scene(gloss), plane_env(), W, H, fp, ro)
    check_clearcoat(img, fp, W, H, gloss)
