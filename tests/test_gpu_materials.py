"""GPU parity for every material branch the reference's inspector can reach
(`src/sources/main.cpp:398-472` sliders; `src/core/Scene.h:53-109` presets), not only the
configurations' materials:

* media: SCATTER (mediumType 2: free flight with xi_3, SampleHG/PhaseHG RT:1195-1222,
  RT:1440-1457) at anisotropy -0.5 / 0 / +0.5, EMISSIVE (mediumType 3, RT:1437-1439, the
  reference's own `tear_glass_emissive` preset, Scene.h:102-108), ABSORB is covered by C4/C5;
* surface emission Le (RT:1509-1510 on continuation hits, RT:1530 on camera hits);
* the Disney lobes the configurations leave at 0: clearcoat with several clearcoatGloss values
  (EvalClearcoat RT:986-1000, SampleGTR1 RT:716-729, R23), sheen / sheenTint (EvalDiffuse
  RT:925-948), anisotropic (GTR2_Aniso / SmithG_GGX_Aniso RT:447-471 with ax != ay) on metal
  and dielectric, specularTint (GetSpecColor RT:420-427);

each in BSDF mode (shadingImportanceSampling_BSDF, RT:1369-1516) and BRDF mode
(shadingImportanceSampling_BRDF, RT:1290-1367), bit for bit against the oracle with equal ray
counts; BSDF mode also through the megakernel.  The object is the bunny on the reference floor
(C2 placement), so camera, NEE, continuation and inside-the-mesh paths all occur.
"""
import numpy as np
import pytest

from helpers import bit_mismatch, frames_for, gpu_render, oracle_render
from rtamd import configs as cf
from rtamd import scene_lib as sl
from rtamd.renderer import RT_FLAG_MEGAKERNEL

pytestmark = pytest.mark.gpu

MATERIAL_CASES = {
    "scatter_fwd": sl.Material(base_color=(1, 1, 1), specular=1.0, transmission=0.95, ior=1.45, roughness=0.05,
                               medium_type=2, medium_color=(0.8, 0.5, 0.3), medium_density=1.5,
                               medium_anisotropy=0.5),
    "scatter_iso": sl.Material(base_color=(1, 1, 1), specular=1.0, transmission=1.0, ior=1.3,
                               medium_type=2, medium_color=(0.3, 0.7, 0.9), medium_density=0.8,
                               medium_anisotropy=0.0),
    "scatter_back": sl.Material(base_color=(1, 1, 1), specular=1.0, transmission=0.9, ior=1.5, roughness=0.2,
                                medium_type=2, medium_color=(0.9, 0.9, 0.6), medium_density=3.0,
                                medium_anisotropy=-0.5),
    "tear_glass_emissive": cf.MATERIALS["tear_glass_emissive"],
    "emissive_surface": sl.Material(emissive=(4.0, 2.5, 1.0), base_color=(0.6, 0.6, 0.6), roughness=0.5,
                                    specular=0.5),
    "clearcoat_gloss0.1": sl.Material(base_color=(0.2, 0.3, 0.8), roughness=0.6, specular=0.5, clearcoat=1.0,
                                      clearcoat_gloss=0.1),
    "clearcoat_gloss0.9": sl.Material(base_color=(0.8, 0.2, 0.1), roughness=0.3, specular=0.5, clearcoat=0.7,
                                      clearcoat_gloss=0.9, metallic=0.3),
    "sheen": sl.Material(base_color=(0.7, 0.2, 0.5), roughness=0.8, specular=0.3, sheen=1.0, sheen_tint=0.6),
    "aniso_metal": sl.Material(base_color=(0.95, 0.64, 0.54), roughness=0.4, specular=1.0, metallic=1.0,
                               anisotropic=0.9),
    "aniso_dielectric": sl.Material(base_color=(0.3, 0.6, 0.3), roughness=0.35, specular=0.8, anisotropic=0.5, ior=1.5,
                                    specular_tint=0.7, sheen=0.3),
    "everything": sl.Material(emissive=(0.2, 0.1, 0.05), base_color=(0.8, 0.7, 0.6), subsurface=0.5, metallic=0.4,
                              specular=0.9, specular_tint=0.5, roughness=0.3, anisotropic=0.6, sheen=0.5,
                              sheen_tint=0.5, clearcoat=0.5, clearcoat_gloss=0.5, ior=1.6, transmission=0.3,
                              medium_type=2, medium_color=(0.5, 0.6, 0.7), medium_density=1.0,
                              medium_anisotropy=0.3),
}


def material_scene(name: str):
    obj = cf.Obj("bunny_4000", MATERIAL_CASES[name], (0, 0, 0), (2.2, -2.5, 3), (2, 2, 2), False)
    return cf.build_scene((cf.FLOOR, obj))


_SCENES = {}


def _scene(name):
    if name not in _SCENES:
        _SCENES[name] = material_scene(name)
    return _SCENES[name]


@pytest.mark.parametrize("mode", ["bsdf", "brdf", "megakernel"])
@pytest.mark.parametrize("name", list(MATERIAL_CASES))
def test_material_branch_matches_oracle(gpu_renderer, env_maps, name, mode):
    sd = _scene(name)
    W, H = 64, 36
    flags = RT_FLAG_MEGAKERNEL if mode == "megakernel" else 0
    fp = cf.frame_params(W, H, enable_bsdf=(mode != "brdf"), flags=flags)
    ro, frames = frames_for(fp, 1, 3)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    frac, diff = bit_mismatch(img, ref)
    assert st["rays"] == cnt["rays"], (name, mode, st["rays"], cnt["rays"])
    assert frac == 0.0, f"{name}/{mode}: {int(diff.sum())} of {W * H} pixels differ"


@pytest.mark.parametrize("env,mis", [(False, True), (True, False)], ids=["sky", "env-nomis"])
@pytest.mark.parametrize("name", ["scatter_fwd", "tear_glass_emissive", "emissive_surface", "everything"])
def test_material_branch_env_switches(gpu_renderer, env_maps, name, env, mis):
    sd = _scene(name)
    W, H = 48, 27
    fp = cf.frame_params(W, H, enable_env_map=env, enable_mis=mis)
    ro, frames = frames_for(fp, 1, 2)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    assert st["rays"] == cnt["rays"]
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("name", ["everything", "scatter_back"])
def test_material_branch_full_hd_frame(gpu_renderer, env_maps, name):
    """One whole 1920x1080 frame (the configurations' size) bit for bit, oracle on the host's
    cores (capped at 16 threads)."""
    import os
    import oracle as orc
    sd = _scene(name)
    W, H = 1920, 1080
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 1)
    try:
        threads = max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        threads = max(1, min(16, os.cpu_count() or 1))
    ref, cnt = orc.render(orc.OracleScene(sd.tri_enc, sd.node_enc, env_maps[0], env_maps[1]), frames, W, H,
                          threads=threads)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    frac, diff = bit_mismatch(img, ref)
    assert st["rays"] == cnt["rays"]
    assert frac == 0.0, f"{name} 1080p: {int(diff.sum())} pixels differ"
    assert np.isfinite(img).mean() > 0.99
