"""CPU: the material cases of tests/test_gpu_materials.py actually reach the branches they name.

For each case the oracle renders the scene twice, once with the material and once with the one
parameter under test neutralised (clearcoat 0, sheen 0, anisotropic 0, emission 0, the medium
switched to another type or anisotropy); the images must differ, so the GPU parity tests of
that case compare a branch that contributes to the image, not dead code.  Small frames
(32x18, 2 frames) keep this in seconds.
"""
import dataclasses

import numpy as np
import pytest

from helpers import frames_for, oracle_render
from rtamd import configs as cf
from test_gpu_materials import MATERIAL_CASES

NEUTRAL = {
    "scatter_fwd": {"medium_anisotropy": 0.0},           # SampleHG/PhaseHG g (RT:1195-1222)
    "scatter_iso": {"medium_type": 1.0},                 # SCATTER -> ABSORB (RT:1434-1457)
    "scatter_back": {"medium_anisotropy": 0.5},
    "tear_glass_emissive": {"medium_type": 0.0},         # EMISSIVE medium term (RT:1437-1439)
    "emissive_surface": {"emissive": (0.0, 0.0, 0.0)},  # Le (RT:1509-1510, RT:1530)
    "clearcoat_gloss0.1": {"clearcoat": 0.0},            # EvalClearcoat / SampleGTR1 (RT:986-1000, 716-729)
    "clearcoat_gloss0.9": {"clearcoat_gloss": 0.1},
    "sheen": {"sheen": 0.0},                             # Fsheen (RT:925-948)
    "aniso_metal": {"anisotropic": 0.0},                 # GTR2_Aniso (RT:447-471)
    "aniso_dielectric": {"specular_tint": 0.0},          # GetSpecColor (RT:420-427)
    "everything": {"sheen_tint": 0.0},
}


def _render(mat, W=32, H=18, **fp_kw):
    obj = cf.Obj("bunny_4000", mat, (0, 0, 0), (2.2, -2.5, 3), (2, 2, 2), False)
    sd = cf.build_scene((cf.FLOOR, obj))
    fp = cf.frame_params(W, H, **fp_kw)
    _, frames = frames_for(fp, 1, 2)
    img, cnt = oracle_render(sd, cf.load_env(), W, H, frames)
    return img, cnt


def test_every_case_has_a_neutral_variant():
    assert set(NEUTRAL) == set(MATERIAL_CASES)


@pytest.mark.parametrize("name", list(MATERIAL_CASES))
def test_case_parameter_reaches_the_image(name):
    mat = MATERIAL_CASES[name]
    img, cnt = _render(mat)
    ref, _ = _render(dataclasses.replace(mat, **NEUTRAL[name]))
    assert cnt["rays"] > 0
    assert np.isfinite(img).mean() > 0.95
    diff = np.any(img.view(np.uint32) != ref.view(np.uint32), axis=-1)
    assert diff.mean() > 0.01, f"{name}: {NEUTRAL[name]} leaves the image unchanged"
