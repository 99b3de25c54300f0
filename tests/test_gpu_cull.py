"""GPU: the traversal's closest-hit culling is exact on an adversarial scene.

tests/cull_cases.py builds a scene where the reference's accepted closest hit (triangle T) lies
several units before the entry of T's own box, and a wall between them is found first by the
near-first traversal.  With the derived bound (cull_eps, rt_render.hip cull_bound_stats) the GPU
image equals the oracle bit for bit; with the bound's eps term forced to 0
(RT_CULL_EPS_SCALE=0, the round-1 margin; a switch only lib/librtamd_dev.so reads) the GPU culls
T's box and returns the wall: the test also checks that this failure shows, so it really
exercises the hole (the near-first child order enters the wall's box before T's).
"""
import numpy as np
import pytest

from cull_cases import old_margin_counterexample
from helpers import bit_mismatch
from rtamd import configs as cf
from rtamd.renderer import RT_FLAG_MEGAKERNEL
from test_cull_bound import cull_frame_params

pytestmark = pytest.mark.gpu


def _render_both(r, env, c, fp, W=8, H=8, n=2):
    import oracle as orc
    ro = cf.rand_origins(n)
    frames = [cf.oracle_frame_params(fp, k + 1, ro[k]) for k in range(n)]
    ref, cnt = orc.render(orc.OracleScene(c["tri_enc"], c["node_enc"], env[0], env[1]), frames, W, H)
    r.set_scene_encoded(c["tri_enc"], c["node_enc"])
    r.set_env(env[0], env[1])
    r.resize(W, H)
    r.set_loop_num(0)
    r.reset_stats()
    st = r.render(fp, ro)
    return r.read_accum(), ref, st, cnt


@pytest.mark.parametrize("flags", [0, RT_FLAG_MEGAKERNEL], ids=["wavefront", "megakernel"])
def test_culling_keeps_the_reference_hit(gpu_renderer, gpu_dev_renderer, env_maps, monkeypatch, flags):
    c = old_margin_counterexample()
    fp = cull_frame_params(c)
    fp.flags = flags
    img, ref, st, cnt = _render_both(gpu_renderer, env_maps, c, fp)
    assert st["rays"] == cnt["rays"]
    assert bit_mismatch(img, ref)[0] == 0.0
    monkeypatch.setenv("RT_CULL_EPS_SCALE", "0")
    same, _, _, _ = _render_both(gpu_renderer, env_maps, c, fp)
    assert bit_mismatch(same, ref)[0] == 0.0, "the release library must ignore RT_CULL_EPS_SCALE"
    bad, _, _, _ = _render_both(gpu_dev_renderer, env_maps, c, fp)
    assert bit_mismatch(bad, ref)[0] > 0.5, "the round-1 margin should lose T on this scene"
    assert np.all(bad[..., 1] > bad[..., 0]), "with the round-1 margin the green wall wins"
