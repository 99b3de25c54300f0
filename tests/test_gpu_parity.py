"""GPU parity: the HIP path tracer against the CPU oracle, bit for bit.

Both sides evaluate the shader's arithmetic in the same fp32 order with the same builtin
definitions (glsl_math.h), so every pixel must match exactly — the fp32 tolerance of
BASELINE.json's north star ("within a stated fp32 tolerance") is here 0 ulp.  The only
admitted deviation is the closest-hit culling of the GPU traversal, which changes nothing
but exact-tie order; the culled and exhaustive GPU paths are both checked.
"""
from types import SimpleNamespace

import numpy as np
import pytest

from helpers import bit_mismatch, frames_for, gpu_render, oracle_render
from rtamd import configs as cf
from rtamd import scene_lib as sl
from rtamd.renderer import RT_FLAG_MEGAKERNEL, RT_FLAG_NO_CULL, RT_FLAG_SORTED_TRAVERSAL

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("flags", [0, RT_FLAG_MEGAKERNEL], ids=["wavefront", "megakernel"])
@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5"])
def test_config_matches_oracle_bitwise(gpu_renderer, env_maps, name, flags):
    sd = cf.config_scene(name)
    W, H = 96, 54
    fp = cf.frame_params(W, H, flags=flags)
    ro, frames = frames_for(fp, 1, 2)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    frac, _ = bit_mismatch(img, ref)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert st["samples"] == cnt["samples"] == W * H * 2
    if not flags & RT_FLAG_MEGAKERNEL:  # shade steps: one per path per pass, each after that path traced 1-2 rays
        assert st["samples"] <= st["path_steps"] <= st["rays"], st
    assert frac == 0.0, f"{name}: {frac:.4%} of pixels differ from the oracle"


def test_pass1_ray_count(gpu_renderer, env_maps):
    """rt_stats.p1_rays (bench.py prices these rays at their 16-B records): without the finisher,
    pass 1 traces the shadow rays and continuations pass 0 queued, so camera + pass-1 rays never
    exceed the total and, with the dragon in view, pass 1 is not empty."""
    from rtamd.renderer import RT_FLAG_NO_FINISH
    sd = cf.config_scene("C3")
    W, H = 96, 54
    fp = cf.frame_params(W, H, flags=RT_FLAG_NO_FINISH)
    ro, frames = frames_for(fp, 1, 2)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    assert bit_mismatch(img, ref)[0] == 0.0 and st["rays"] == cnt["rays"]
    assert 0 < st["p1_rays"] and st["samples"] + st["p1_rays"] <= st["rays"], st


def test_no_cull_matches_too(gpu_renderer, env_maps):
    sd = cf.config_scene("C3")
    W, H = 64, 36
    fp = cf.frame_params(W, H, flags=RT_FLAG_NO_CULL)
    ro, frames = frames_for(fp, 1, 1)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    img, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_encoded_aos_entry_point(gpu_renderer, env_maps):
    sd = cf.config_scene("C2")
    W, H = 48, 32
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 1)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    img, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro, encoded=True)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_frames_in_flight_capacity_does_not_change_the_image(gpu_renderer, env_maps):
    """Frames in flight are blended in frame order: 1 frame per wavefront (tiny path-state
    budget) and all frames at once give the same bits, and both equal the oracle."""
    sd = cf.config_scene("C3")
    W, H = 64, 36
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 3)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    gpu_renderer.set_max_paths(W * H)  # -> one frame in flight
    try:
        img1, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    finally:
        gpu_renderer.set_max_paths(0)  # the library default
    img3, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    assert bit_mismatch(img1, ref)[0] == 0.0
    assert bit_mismatch(img3, ref)[0] == 0.0


@pytest.mark.parametrize("width,rebuild", [("4", "1"), ("4", "0"), ("2", "1")],
                         ids=["bvh4-rebuilt", "bvh4-reflevels", "bvh2"])
def test_exact_distance_ties_follow_reference_order(gpu_dev_renderer, env_maps, monkeypatch, width, rebuild):
    """Two copies of the bunny at the same place with different materials: every hit on it is an
    exact distance tie between two triangles in different leaves.  The reference keeps the one
    its near-first DFS reaches first; the 4-wide traversal visits leaves in another order and
    must resolve each tie to that same triangle (tie_wins), the binary one by construction."""
    twin = cf.Obj("bunny_4000", "golden", (0, 0, 0), (2.2, -2.5, 3), (2, 2, 2), False)
    sd = cf.build_scene((cf.FLOOR, cf.BUNNY, twin))
    W, H = 64, 36
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 1)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    monkeypatch.setenv("RT_BVH_WIDTH", width)
    monkeypatch.setenv("RT_REBUILD", rebuild)
    img, st = gpu_render(gpu_dev_renderer, sd, env_maps, W, H, fp, ro)
    assert st["rays"] == cnt["rays"]
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("name", ["C3", "C5"])
def test_reference_internal_levels_match_too(gpu_dev_renderer, env_maps, monkeypatch, name):
    """RT_REBUILD=0 (lib/librtamd_dev.so) collapses the reference's own internal nodes instead of the SAH levels rebuilt
    over its leaves (rebuild_over_leaves): both reach exactly the leaves whose boxes the ray hits,
    so both images equal the oracle, and the rebuilt tree takes fewer node steps per ray."""
    from rtamd.renderer import RT_FLAG_COUNT_VISITS
    sd = cf.config_scene(name)
    W, H = 64, 36
    fp = cf.frame_params(W, H, flags=RT_FLAG_COUNT_VISITS)
    ro, frames = frames_for(fp, 1, 1)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    visits = {}
    for rebuild in ("0", "1"):
        monkeypatch.setenv("RT_REBUILD", rebuild)
        img, st = gpu_render(gpu_dev_renderer, sd, env_maps, W, H, fp, ro)
        assert bit_mismatch(img, ref)[0] == 0.0, rebuild
        visits[rebuild] = st["internal_pops"] / st["rays"]
    assert visits["1"] < visits["0"], visits


def test_binary_wavefront_traversal_matches(gpu_dev_renderer, env_maps, monkeypatch):
    """RT_BVH_WIDTH=2 (lib/librtamd_dev.so) keeps the wavefront trace on the binary tree (reference visit order)."""
    sd = cf.config_scene("C3")
    W, H = 64, 36
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 2)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    monkeypatch.setenv("RT_BVH_WIDTH", "2")
    img, _ = gpu_render(gpu_dev_renderer, sd, env_maps, W, H, fp, ro)
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("env,mis", [(True, True), (True, False), (False, True)], ids=["env-mis", "env-nomis", "sky"])
@pytest.mark.parametrize("name", ["C2", "C3", "C4", "C5"])
def test_brdf_mode_matches_oracle_bitwise(gpu_renderer, env_maps, name, env, mis):
    """enableBSDF = false: shadingImportanceSampling_BRDF (RT:1290-1367) on the wavefront path."""
    sd = cf.config_scene(name)
    W, H = 64, 36
    fp = cf.frame_params(W, H, enable_bsdf=False, enable_env_map=env, enable_mis=mis)
    ro, frames = frames_for(fp, 1, 2)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_megakernel_rejects_brdf_mode(gpu_renderer, env_maps):
    sd = cf.config_scene("C2")
    fp = cf.frame_params(32, 32, enable_bsdf=False, flags=RT_FLAG_MEGAKERNEL)
    with pytest.raises(RuntimeError, match="wavefront path only"):
        gpu_render(gpu_renderer, sd, env_maps, 32, 32, fp, cf.rand_origins(1))


@pytest.mark.parametrize("env,mis", [(False, True), (True, False)], ids=["sky", "env-nomis"])
def test_bsdf_mode_env_and_mis_switches(gpu_renderer, env_maps, env, mis):
    """enableEnvMap / enableMultiImportantSample off in BSDF mode (RT:1383-1405, 1483-1506)."""
    sd = cf.config_scene("C4")
    W, H = 64, 36
    fp = cf.frame_params(W, H, enable_env_map=env, enable_mis=mis)
    ro, frames = frames_for(fp, 1, 2)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    img, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("bsdf", [1, 0], ids=["bsdf", "brdf"])
@pytest.mark.parametrize("finish", ["off", "pass1", "pass2", "pass8"])
@pytest.mark.parametrize("name", ["C3", "C4"])
def test_path_persistent_finisher_matches_oracle(gpu_renderer, env_maps, name, finish, bsdf):
    """wf_finish (one lane per remaining path, trace + shade until the path ends) against the
    pure pass-by-pass wavefront and the oracle, for every pass it can take over from: the image
    bits and the ray count are unchanged.  C4's glass keeps paths alive through refraction."""
    from rtamd.renderer import RT_FLAG_FINISH, RT_FLAG_NO_FINISH
    sd = cf.config_scene(name)
    W, H = 80, 48
    flags = RT_FLAG_NO_FINISH if finish == "off" else RT_FLAG_FINISH
    fp = cf.frame_params(W, H, flags=flags)
    fp.enable_bsdf = bsdf
    ro, frames = frames_for(fp, 1, 2)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    if finish != "off":
        gpu_renderer.set_finish(int(finish[4:]), 1 << 30)
    try:
        img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    finally:
        gpu_renderer.set_finish(2, 8 << 20)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("name", ["C3", "C4"])
def test_lane_quads_move_overflow_stacks(gpu_dev_renderer, env_maps, monkeypatch, name):
    """The lane-quad tails (wf_finish and the small passes' wf_trace) copy each path's
    stack to its quad, LDS entries and overflow entries alike.  With one LDS entry per lane
    (RT_LDS_STACK=1, dev library) nearly every stacked subtree is in the overflow columns when a
    wave moves its paths, and the image and the ray count still equal the oracle's."""
    from rtamd.renderer import RT_FLAG_FINISH
    sd = cf.config_scene(name)
    W, H = 80, 48
    fp = cf.frame_params(W, H, flags=RT_FLAG_FINISH)
    ro, frames = frames_for(fp, 1, 1)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    monkeypatch.setenv("RT_LDS_STACK", "1")
    img, st = gpu_render(gpu_dev_renderer, sd, env_maps, W, H, fp, ro)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


def _deep_chain_scene(depth=64):
    """A BVH at the library's depth limit (rt_set_scene: RT_ERR_LIMIT beyond 64 levels): `depth`
    stacked triangles in planes z = const facing the camera, in a chain tree whose level i has the
    farthest remaining triangle as one child and the rest as the other, so a ray through the stack
    enters the near chain first and pushes a far child on every level (Triangle_encoded /
    BVHNode_encoded, src/core/Triangle.h:28-39, src/core/BVH.h:17-21)."""
    n = depth
    mats = [cf.MATERIALS["brown_glass"].texels(), cf.MATERIALS["jade"].texels()]
    tri = np.zeros((n, 14, 3), np.float32)
    box = []
    for t in range(n):  # t = 0 farthest (z = -3.15) ... n - 1 nearest (z = 0)
        z = np.float32(-0.05 * (n - 1 - t))
        dx, dy = 0.03 * np.sin(t), 0.03 * np.cos(t)
        p = np.array([(-7.5 + dx, -4.2 + dy, z), (7.6 + dx, -4.0 + dy, z), (0.1 + dx, 5.5 + dy, z)], np.float32)
        tri[t, 0:3] = p
        tri[t, 3:6] = (0.0, 0.0, 1.0)
        tri[t, 6:14] = mats[t % 2].reshape(8, 3)
        box.append((p.min(0), p.max(0)))
    nodes = np.zeros((2 * n, 4, 3), np.float32)

    def leaf(j, t):
        nodes[j, 1] = (1, t, 0)
        nodes[j, 2], nodes[j, 3] = box[t]

    # internal level i (1-based, root = node 1) is node 2i-1: left = the far leaf 2i holding
    # triangle i-1, right = the chain 2i+1 (on the last level the leaf of the nearest triangle)
    for i in range(n - 1, 0, -1):
        j, lj, rj = 2 * i - 1, 2 * i, 2 * i + 1
        leaf(lj, i - 1)
        if i == n - 1:
            leaf(rj, n - 1)
        lo = np.min([b[0] for b in box[i - 1:]], 0)
        hi = np.max([b[1] for b in box[i - 1:]], 0)
        nodes[j, 0] = (lj, rj, 0)
        nodes[j, 2], nodes[j, 3] = lo, hi
    return tri, nodes


def test_bvh_deeper_than_the_limit_is_refused(gpu_renderer):
    """65 levels: rt_set_scene fails with RT_ERR_LIMIT (rt_abi.h), it does not render wrongly."""
    tri, nodes = _deep_chain_scene(65)
    with pytest.raises(RuntimeError) as e:
        gpu_renderer.set_scene_encoded(tri, nodes)
    assert "deeper than 64" in str(e.value)


@pytest.mark.parametrize("dev", [False, True])
def test_deepest_bvh_renders_and_moves_whole_stacks(gpu_renderer, gpu_dev_renderer, env_maps, monkeypatch, dev):
    """A chain BVH at the depth limit renders bit-exact, including its lane-quad moves:
    the moves copy a path's whole stack, up to the scene's deepest (KParams::stack_cap), where they
    used to stop at LDS + 64 entries and the host refused any scene deeper than that.  The dev
    variant keeps the reference's own chain as the 4-wide tree (RT_REBUILD=0: 3 pushes per 4-wide
    node, ~64 stacked entries) with one LDS entry per lane (RT_LDS_STACK=1), so nearly the whole
    stack sits in the overflow columns when the small passes' tails and the finisher move it."""
    from rtamd.renderer import RT_FLAG_FINISH
    tri, nodes = _deep_chain_scene(64)
    W, H = 80, 48
    cam = sl.camera(-90.0, 0.0, cf.CAMERA_ZOOM, float(np.float32(W) / np.float32(H)))
    fp = cf.frame_params(W, H, flags=RT_FLAG_FINISH, front=cam["front"], right=cam["right"], up=cam["up"],
                         left_bottom_corner=cam["left_bottom_corner"], half_h=cam["half_h"], half_w=cam["half_w"])
    ro, frames = frames_for(fp, 1, 2)
    import oracle as orc
    ref, cnt = orc.render(orc.OracleScene(tri, nodes, env_maps[0], env_maps[1]), frames, W, H)
    r = gpu_renderer
    if dev:
        monkeypatch.setenv("RT_LDS_STACK", "1")
        monkeypatch.setenv("RT_REBUILD", "0")
        r = gpu_dev_renderer
    img, st = gpu_render(r, SimpleNamespace(tri_enc=tri, node_enc=nodes), env_maps, W, H, fp, ro, encoded=True)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


def _level_camera(W, H, yaw=-90.0):
    """The default camera turned level (pitch 0, Camera.h:160-174): Front.y = sin(0) = 0, so Right.y
    = 0 and Up = (0, u, 0), and the camera ray of every pixel of the middle row of an odd height
    (v = 0.5: LBC.y = -halfH*Up.y, plus (0.5*2*halfH)*Up.y) has a y component of exactly 0."""
    cam = sl.camera(yaw, 0.0, cf.CAMERA_ZOOM, float(np.float32(W) / np.float32(H)))
    return cf.frame_params(W, H, front=cam["front"], right=cam["right"], up=cam["up"],
                           left_bottom_corner=cam["left_bottom_corner"], half_h=cam["half_h"],
                           half_w=cam["half_w"])


def _camera_dirs(fp, W, H):
    """wf_camera's operations (RT:1527 before normalize, fp32, left to right): the unnormalised
    camera directions, (H, W, 3); a zero component stays zero through normalize."""
    f = np.float32
    px, py = np.meshgrid(np.arange(W, dtype=f), np.arange(H, dtype=f))
    u = (px + f(0.5)) / f(W)
    v = (py + f(0.5)) / f(H)
    a = (u * f(2.0)) * f(fp.half_w)
    b = (v * f(2.0)) * f(fp.half_h)
    lbc, right, up = (np.asarray(x, f) for x in (fp.left_bottom_corner, fp.right, fp.up))
    return np.stack([(lbc[k] + a * right[k]) + b * up[k] for k in range(3)], axis=-1)


@pytest.mark.parametrize("small", [True, False], ids=["finisher-static", "bulk-kernels"])
def test_zero_direction_component_rays_match_oracle(gpu_renderer, env_maps, small):
    """Rays with an exactly zero direction component take the literal slab of RT:309-310 (1/d =
    +-inf; tl_qnode_keys / coop_box).  Its per-axis min / max turns a QNode's empty slot (the
    inverted box lo = +inf, hi = -inf) into an infinite box, so that path must test the slot's ref:
    round 4 (ccd9513) entered such a slot, i.e. fetched QNode 0x7fffffff (Q_EMPTY), far outside
    the array — the hipErrorIllegalAddress of gpurun_out/fast1/tests.log.  No other
    test had such rays (every configuration's camera has pitch -14).  A level camera over C3 gives
    the middle row of an odd-height frame camera rays with d.y = 0, which cross the dragon's tree
    (4-wide nodes with fewer than four children sit at every level above its leaves).  Both trace
    kernel families run it: the one-frame / small-pass kernels with the finisher's lane quads, and
    the bulk kernels (finisher slot limit 1).  The image and the ray count equal the oracle's."""
    sd = cf.config_scene("C3")
    W, H = 64, 37
    fp = _level_camera(W, H)
    d = _camera_dirs(fp, W, H)
    assert np.all(d[(H - 1) // 2, :, 1] == 0.0) and np.count_nonzero(d[..., 1] == 0.0) == W
    ro, frames = frames_for(fp, 1, 2)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    if not small:
        r.set_finish(2, 1)
    try:
        img, st = gpu_render(r, sd, env_maps, W, H, fp, ro)
    finally:
        r.set_finish(2, 8 << 20)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0
    # the row's camera rays hit the scene (they traverse, not just miss the root box)
    assert np.any(np.abs(ref[(H - 1) // 2] - ref[0]).sum(axis=-1) > 0)


def test_sorted_traversal_flag_is_accepted(gpu_renderer, env_maps):
    """RT_FLAG_SORTED_TRAVERSAL (ABI 4) has no effect since ABI 5 (the octant-ordered traversal it
    switched off was removed): a call with it renders the same image as one without."""
    sd = cf.config_scene("C3")
    W, H = 48, 32
    ro, frames = frames_for(cf.frame_params(W, H), 1, 1)
    a, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, cf.frame_params(W, H), ro)
    b, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, cf.frame_params(W, H, flags=RT_FLAG_SORTED_TRAVERSAL), ro)
    assert bit_mismatch(a, b)[0] == 0.0


@pytest.mark.parametrize("small", [True, False], ids=["small-pass-kernels", "bulk-kernels"])
@pytest.mark.parametrize("W,H,n", [(3, 2, 1), (11, 7, 3), (40, 23, 2)])
def test_segment_claims_on_tiny_passes(gpu_renderer, env_maps, W, H, n, small):
    """Round 5: the trace passes claim their rays from 8 queue segments (one counter line each; the
    small passes after their static shares), and a wave moves on when its segment is exhausted.
    Passes of 0-7 rays leave segments empty and make every wave walk all 8; frames of 6 to 920
    pixels, with the bulk kernels (finisher slot limit 1) and the small-pass ones (finisher off so
    every pass is a wavefront pass): image and ray count equal the oracle's."""
    from rtamd.renderer import RT_FLAG_NO_FINISH
    sd = cf.config_scene("C4")  # glass: paths that live to the last bounces
    fp = cf.frame_params(W, H, flags=0 if not small else RT_FLAG_NO_FINISH)
    ro, frames = frames_for(fp, 1, n)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    if not small:
        r.set_finish(2, 1)
    try:
        img, st = gpu_render(r, sd, env_maps, W, H, fp, ro)
    finally:
        r.set_finish(2, 8 << 20)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert st["samples"] == W * H * n
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("name,W,H,n,small,bsdf,env", [
    ("C3", 24, 16, 256, False, 1, True),   # 128 frames per group: 16 pixels per block-iteration
    ("C3", 20, 13, 130, False, 1, False),  # 65 frames: pixels straddle block-iterations; sky misses
    ("C4", 16, 11, 200, True, 1, True),    # small-pass kernels (no records: every frame computes its hit); glass
    ("C3", 16, 12, 160, False, 0, True),   # BRDF integrator (the record's geometry only)
    ("C4", 16, 11, 192, False, 1, True),   # glass: refraction lobe (G1V) and absorbing medium in the records
    ("C2", 20, 12, 128, False, 1, True),   # jade: diffuse / fake-subsurface lobe (FV)
], ids=["C3-128", "C3-65-sky", "C4-small", "C3-brdf", "C4-bulk", "C2-bulk"])
def test_camera_hit_records_match_oracle(gpu_renderer, env_maps, name, W, H, n, small, bsdf, env):
    """Round 5: with at least 64 frames per bulk group the camera pass's shade (wf_shade<..., CAM>)
    computes each pixel's camera hit (geometry, emission, BSDF frame and the V-only BSDF terms, or
    the miss colour) once per block-iteration into LDS and the frames read it there.  Frames of a
    pixel shade the same hit, so the image and ray count stay the oracle's, bit for bit, in both
    integrators; the small-pass kernels, which keep no records, are checked at the same sizes."""
    from rtamd.renderer import RT_FLAG_NO_FINISH
    sd = cf.config_scene(name)
    fp = cf.frame_params(W, H, flags=RT_FLAG_NO_FINISH if small else 0, enable_env_map=env)
    fp.enable_bsdf = bsdf
    ro, frames = frames_for(fp, 1, n)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    if not small:
        r.set_finish(2, 1)
    try:
        img, st = gpu_render(r, sd, env_maps, W, H, fp, ro)
    finally:
        r.set_finish(2, 8 << 20)
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert st["samples"] == W * H * n
    assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("name", ["C3", "C4"])
def test_split_queues_in_every_pass_match(gpu_dev_renderer, env_maps, monkeypatch, name):
    """Split queues (a bulk pass's shadow rays traced by the any-hit wf_trace<..., 2>,
    its continuations by <..., 1>) leave the image and the ray count unchanged whichever passes use
    them: RT_SPLIT_KINDS=0 (one queue of both kinds in every pass), RT_SPLIT_PASSES=8 (split in
    every secondary pass) and the default (passes 1-5) render the bulk path (frame groups of 9.4 M
    path slots, above the finisher's budget) bit-identically, and an 8x8 window of the default
    equals the oracle (dev library switches)."""
    sd = cf.config_scene(name)
    W, H, NF = 256, 144, 512
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, NF)
    out = {}
    try:
        for key, env in (("default", {}), ("one_queue", {"RT_SPLIT_KINDS": "0"}), ("all_passes", {"RT_SPLIT_PASSES": "8"})):
            for k in ("RT_SPLIT_KINDS", "RT_SPLIT_PASSES"):
                monkeypatch.delenv(k, raising=False)
            for k, v in env.items():
                monkeypatch.setenv(k, v)
            gpu_dev_renderer.set_max_paths(NF * W * H)  # one launch of two 256-frame groups
            out[key] = gpu_render(gpu_dev_renderer, sd, env_maps, W, H, fp, ro)
            assert out[key][1]["launches"] == 1 and out[key][1]["finish_steps"] == 0, out[key][1]
    finally:
        for k in ("RT_SPLIT_KINDS", "RT_SPLIT_PASSES"):
            monkeypatch.delenv(k, raising=False)
        gpu_dev_renderer.set_max_paths(0)  # the library default again (a session fixture)
    img, st = out["default"]
    for key in ("one_queue", "all_passes"):
        assert out[key][1]["rays"] == st["rays"], (key, out[key][1], st)
        assert bit_mismatch(out[key][0], img)[0] == 0.0, key
    x0, y0 = 120, 56  # the object's silhouette region
    ref, cnt = oracle_render(sd, env_maps, W, H, frames, x0=x0, y0=y0, w=8, h=8)
    assert bit_mismatch(img[y0:y0 + 8, x0:x0 + 8], ref)[0] == 0.0
