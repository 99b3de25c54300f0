"""The packet traversal (wf_trace_pkt, round 6) against the oracle, bit for bit.

The 64 rays of a wave traverse the 4-wide tree together: scalar node loads, per-lane
box tests and cull limits, a wave-uniform stack holding each lane's own entry distance, per-lane
leaf tests.  Every lane still tests exactly the leaves whose boxes its ray hits, so images and ray
counts equal the oracle's.  The development library selects it per pass (RT_PKT_PASSES, bit p =
pass p) for the bulk kernels (finisher slot limit 1, as at the bench's frame groups); these tests
run every pass with it, over the configurations, the integrators, culling off, rays with a zero
direction component (the literal slab: no wave-uniform octant), exact distance ties and a BVH at
the depth limit (64-entry stacks, overflow columns).
"""
from types import SimpleNamespace

import numpy as np
import pytest

from helpers import bit_mismatch, frames_for, gpu_render, oracle_render
from rtamd import configs as cf

pytestmark = pytest.mark.gpu

ALL_PASSES = "0x1ff"


def _render_pkt(r, monkeypatch, sd, env, W, H, fp, ro, passes=ALL_PASSES, encoded=False):
    monkeypatch.setenv("RT_PKT_PASSES", passes)
    r.set_finish(2, 1)  # every frame group on the bulk kernels
    try:
        return gpu_render(r, sd, env, W, H, fp, ro, encoded=encoded)
    finally:
        r.set_finish(2, 8 << 20)


@pytest.mark.parametrize("name,W,H,n", [("C2", 32, 18, 64), ("C3", 48, 27, 64), ("C4", 32, 18, 64),
                                        ("C5", 32, 18, 32), ("C3", 96, 54, 2)])
def test_packet_traversal_matches_oracle(gpu_dev_renderer, env_maps, monkeypatch, name, W, H, n):
    sd = cf.config_scene(name)
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, n)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = _render_pkt(gpu_dev_renderer, monkeypatch, sd, env_maps, W, H, fp, ro)
    assert st["finish_steps"] == 0
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("variant", ["no-cull", "brdf", "sky", "passes-0-1"])
def test_packet_traversal_variants(gpu_dev_renderer, env_maps, monkeypatch, variant):
    from rtamd.renderer import RT_FLAG_NO_CULL
    sd = cf.config_scene("C4" if variant == "brdf" else "C3")
    W, H, n = 32, 18, 64
    kw = {"no-cull": dict(flags=RT_FLAG_NO_CULL), "brdf": dict(enable_bsdf=False),
          "sky": dict(enable_env_map=False), "passes-0-1": {}}[variant]
    fp = cf.frame_params(W, H, **kw)
    ro, frames = frames_for(fp, 1, n)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = _render_pkt(gpu_dev_renderer, monkeypatch, sd, env_maps, W, H, fp, ro,
                          passes="0x3" if variant == "passes-0-1" else ALL_PASSES)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_packet_traversal_zero_direction_rays(gpu_dev_renderer, env_maps, monkeypatch):
    """A level camera: the middle row's camera rays have d.y = 0 (1/d infinite), so their packets
    have no wave-uniform octant and take the literal slab per lane."""
    from test_gpu_parity import _camera_dirs, _level_camera
    sd = cf.config_scene("C3")
    W, H = 64, 37
    fp = _level_camera(W, H)
    assert np.count_nonzero(_camera_dirs(fp, W, H)[..., 1] == 0.0) == W
    ro, frames = frames_for(fp, 1, 4)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = _render_pkt(gpu_dev_renderer, monkeypatch, sd, env_maps, W, H, fp, ro)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_packet_traversal_exact_ties(gpu_dev_renderer, env_maps, monkeypatch):
    """Two coincident bunnies with different materials: every hit on them is an exact distance tie,
    resolved by tie_wins whatever order the packet visits the leaves in."""
    twin = cf.Obj("bunny_4000", "golden", (0, 0, 0), (2.2, -2.5, 3), (2, 2, 2), False)
    sd = cf.build_scene((cf.FLOOR, cf.BUNNY, twin))
    W, H = 32, 18
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 16)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = _render_pkt(gpu_dev_renderer, monkeypatch, sd, env_maps, W, H, fp, ro)
    assert st["rays"] == cnt["rays"]
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("rebuild", ["1", "0"])
def test_packet_traversal_deepest_bvh(gpu_dev_renderer, env_maps, monkeypatch, rebuild):
    """The chain BVH at the depth limit (test_gpu_parity._deep_chain_scene): with the reference's
    own levels (RT_REBUILD=0) a packet's stack grows three entries per 4-wide node, into the
    overflow columns (RT_LDS_STACK=1)."""
    import oracle as orc
    from rtamd import scene_lib as sl
    from test_gpu_parity import _deep_chain_scene
    tri, nodes = _deep_chain_scene(64)
    W, H = 32, 18
    cam = sl.camera(-90.0, 0.0, cf.CAMERA_ZOOM, float(np.float32(W) / np.float32(H)))
    fp = cf.frame_params(W, H, front=cam["front"], right=cam["right"], up=cam["up"],
                         left_bottom_corner=cam["left_bottom_corner"], half_h=cam["half_h"], half_w=cam["half_w"])
    ro, frames = frames_for(fp, 1, 8)
    ref, cnt = orc.render(orc.OracleScene(tri, nodes, env_maps[0], env_maps[1]), frames, W, H)
    monkeypatch.setenv("RT_REBUILD", rebuild)
    monkeypatch.setenv("RT_LDS_STACK", "1")
    img, st = _render_pkt(gpu_dev_renderer, monkeypatch, SimpleNamespace(tri_enc=tri, node_enc=nodes), env_maps,
                          W, H, fp, ro, encoded=True)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0
