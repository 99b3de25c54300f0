"""GPU tests of the C-ABI semantics around the kernel (include/rt_abi.h): progressive
accumulation across calls, history written by the host, the maxIterations cap (R12),
material updates, odd frame / tile sizes, an empty scene, and the multi-rank tile split with
the device-side frame assembly.  Every image is checked bit for bit against the oracle."""
import numpy as np
import pytest

from helpers import bit_mismatch, frames_for, gpu_render, oracle_render
from rtamd import configs as cf
from rtamd import scene_lib as sl
from rtamd import tiling
from rtamd.renderer import RT_GATHER_PEER, RT_GATHER_RCCL

pytestmark = pytest.mark.gpu


def _scene_from(s: sl.Scene) -> cf.SceneData:
    tri, nodes = s.encode()
    return cf.SceneData("custom", s.counts(), tri, nodes, s.export_soa(), s.nodes(), [])


def test_progressive_accumulation_across_calls(gpu_renderer, env_maps):
    """Frames 1-2 in one call and 3-5 in the next == frames 1-5 (main.cpp:175-200 LoopNum)."""
    sd = cf.config_scene("C2")
    W, H = 48, 32
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 5)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    gpu_render(r, sd, env_maps, W, H, fp, ro[:2])
    r.render(fp, ro[2:])
    assert r.loop_num == 5
    assert bit_mismatch(r.read_accum(), ref)[0] == 0.0


def test_host_written_history_and_loop_num(gpu_renderer, env_maps):
    """rt_write_accum + rt_set_loop_num resume a progressive render from a given history."""
    sd = cf.config_scene("C3")
    W, H = 40, 24
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 4)
    hist, _ = oracle_render(sd, env_maps, W, H, frames[:2])
    ref, _ = oracle_render(sd, env_maps, W, H, frames[2:], accum=hist)
    img, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro[2:], accum=hist, loop_num=2)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_max_iterations_caps_progression(gpu_renderer, env_maps):
    """maxIterations = 3: LoopNum stops at 3 and frames at the cap trace nothing (R12)."""
    sd = cf.config_scene("C2")
    W, H = 32, 32
    fp = cf.frame_params(W, H, max_iterations=3)
    ro = cf.rand_origins(6)
    # host logic of main.cpp:175-178 over six frames: loop 1, 2 traced, then 3, 3, 3, 3 untraced
    frames, loop = [], 0
    for k in range(6):
        if loop < 3:
            loop += 1
        if loop < 3:
            frames.append(cf.oracle_frame_params(fp, loop, ro[k]))
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    assert gpu_renderer.loop_num == 3
    assert st["samples"] == cnt["samples"] == 2 * W * H
    assert bit_mismatch(img, ref)[0] == 0.0


def test_update_materials_matches_reencoded_scene(gpu_renderer, env_maps):
    """rt_update_materials (RefreshTriangleMaterial) == re-encoding the scene with the material."""
    s = sl.Scene()
    for o in cf.CONFIGS["C2"].objects:
        s.add_mesh(cf.load_mesh(o.mesh), cf.MATERIALS[o.material], o.rotate, o.translate, o.scale, o.smooth)
    s.build_bvh(8)
    before = _scene_from(s)
    n = before.counts["n_triangles"]
    new = cf.MATERIALS["golden"]
    first, count = n // 3, n // 2  # a post-BVH range (rt_abi.h: indices after the BVH sort)
    s.set_material(first, count, new)
    after = _scene_from(s)
    W, H = 48, 32
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 2)
    ref, _ = oracle_render(after, env_maps, W, H, frames)
    r = gpu_renderer
    r.set_scene_soa(before.soa, before.nodes)
    r.update_materials(first, count, new.texels())
    r.set_env(env_maps[0], env_maps[1])
    r.resize(W, H)
    r.set_loop_num(0)
    r.render(fp, ro)
    assert bit_mismatch(r.read_accum(), ref)[0] == 0.0


@pytest.mark.parametrize("W,H,tile", [(37, 23, 16), (70, 9, 32), (1, 1, 8)])
def test_odd_frame_and_tile_sizes(gpu_renderer, env_maps, W, H, tile):
    sd = cf.config_scene("C4")
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 2)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    img, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro, tile=tile)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_empty_scene_renders_the_environment(gpu_renderer, env_maps):
    s = sl.Scene()
    s.build_bvh(8)
    sd = _scene_from(s)
    W, H = 32, 16
    for env in (True, False):
        fp = cf.frame_params(W, H, enable_env_map=env)
        ro, frames = frames_for(fp, 1, 1)
        ref, _ = oracle_render(sd, env_maps, W, H, frames)
        img, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
        assert bit_mismatch(img, ref)[0] == 0.0


@pytest.mark.parametrize("assign", ["modulo", "balanced"])
@pytest.mark.parametrize("world", [2, 3])
def test_tile_split_and_device_assembly(gpu_renderer, env_maps, world, assign):
    """Ranks r = 0..world-1 render their interleaved tiles (one context each, as one process per
    GPU would); the rank-major concatenation of their device tile buffers, un-permuted by
    rt_assemble_frame on the device, is the single-rank frame bit for bit (and the oracle's)."""
    import torch
    from rtamd.renderer import Renderer
    sd = cf.config_scene("C3")
    W, H, T = 80, 45, 16
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 2)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    owner = None
    if assign == "balanced":  # bench.py's cost-balanced owner map (rt_tile_costs + tiling.balance)
        r0 = gpu_renderer
        r0.set_scene_soa(sd.soa, sd.nodes)
        r0.set_env(*env_maps)
        r0.resize(W, H, tile=T)
        before = r0.read_accum()
        costs = r0.tile_costs(fp, ro[:1])
        assert np.array_equal(costs, r0.tile_costs(fp, ro[:1])) and costs.min() > 0
        assert r0.loop_num == 0 and np.array_equal(r0.read_accum(), before)  # the probe leaves no trace
        owner = tiling.balance(costs, world)
        assert not np.array_equal(owner, tiling.modulo_owners(W, H, T, T, world))
    parts = []
    ctxs = [gpu_renderer] + [Renderer(0) for _ in range(world - 1)]
    try:
        for rank, r in enumerate(ctxs):
            gpu_render(r, sd, env_maps, W, H, fp, ro, tile=T, rank=rank, world=world, owner=owner)
            info = r.accum_device()
            buf = torch.empty(info["bytes"] // 4, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()  # buf allocated on torch's stream, copied on the ctx stream
            r.copy_accum_device(buf.data_ptr(), info["bytes"])
            r.synchronize()
            parts.append(buf)
        gathered = torch.cat(parts)
        torch.cuda.synchronize()
        frame = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
        ctxs[0].assemble_frame(gathered.data_ptr(), world, frame.data_ptr())
        torch.cuda.synchronize()
        img = frame.cpu().numpy().reshape(H, W, 3)
        mlt = tiling.max_local_tiles(W, H, T, T, world, owner)
        host = tiling.assemble(gathered.cpu().numpy().reshape(world, mlt, T, T, 4), W, H, T, T, world, owner)
    finally:
        for r in ctxs[1:]:
            r.close()
    assert bit_mismatch(img, ref)[0] == 0.0
    assert bit_mismatch(host[..., :3], ref)[0] == 0.0


def test_single_process_gather(gpu_renderer, env_maps):
    """rt_gather: three rank contexts (one device here; peer copies between GPUs on a node)
    render their tiles asynchronously; the gathered frame equals the oracle bit for bit, and a
    context that is not rank r of the world is refused."""
    from rtamd.renderer import Renderer
    sd = cf.config_scene("C2")
    W, H, T, world = 72, 40, 16, 3
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 3)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    ctxs = [gpu_renderer] + [Renderer(0) for _ in range(world - 1)]
    try:
        for rank, r in enumerate(ctxs):
            r.set_scene_soa(sd.soa, sd.nodes)
            r.set_env(env_maps[0], env_maps[1])
            r.resize(W, H, tile=T, rank=rank, world=world)
            r.set_loop_num(0)
            r.clear_accum()
            r.render_async(fp, ro)  # no synchronisation: rt_gather orders the copies itself
        img = Renderer.gather(ctxs)
        assert ctxs[0].gather_transport() == RT_GATHER_PEER  # (contexts sharing a device)
        with pytest.raises(RuntimeError, match="rank r"):
            Renderer.gather([ctxs[1], ctxs[0], ctxs[2]])
        with pytest.raises(RuntimeError, match="one device per context"):
            Renderer.gather(ctxs, transport=RT_GATHER_RCCL)
    finally:
        for r in ctxs[1:]:
            r.close()
    assert bit_mismatch(img, ref)[0] == 0.0


def test_single_process_gather_rccl(gpu_renderer, env_maps):
    """rt_gather over RCCL: one context per device (every visible device, up to
    8), each rendering its rank's tiles; the communicators come from ncclCommInitAll, every rank
    sends its tiles to rank 0 in one group.  On a one-GPU box that is a world of one (rank 0 sends
    to itself); the frame equals the oracle bit for bit and a second gather reuses the
    communicators."""
    import torch
    from rtamd.renderer import Renderer
    sd = cf.config_scene("C2")
    world = max(1, min(8, torch.cuda.device_count()))
    W, H, T = 72, 40, 16
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 2)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    ctxs = [gpu_renderer] + [Renderer(d) for d in range(1, world)]
    try:
        for rank, r in enumerate(ctxs):
            r.set_scene_soa(sd.soa, sd.nodes)
            r.set_env(env_maps[0], env_maps[1])
            r.resize(W, H, tile=T, rank=rank, world=world)
            r.set_loop_num(0)
            r.clear_accum()
            r.render_async(fp, ro)
        img = Renderer.gather(ctxs)
        assert ctxs[0].gather_transport() == RT_GATHER_RCCL
        img2 = Renderer.gather(ctxs, transport=RT_GATHER_RCCL)
        peer = Renderer.gather(ctxs, transport=RT_GATHER_PEER)
    finally:
        for r in ctxs[1:]:
            r.close()
    assert bit_mismatch(img, ref)[0] == 0.0
    assert np.array_equal(img, img2) and np.array_equal(img, peer)


def test_path_budget_beyond_device_memory_falls_back(env_maps):
    """rt_set_max_paths: a budget larger than HBM (1024 frames of 1080p = 458 GB) runs fewer
    frames per launch; the image equals a run with a small budget bit for bit."""
    from rtamd.renderer import Renderer
    sd = cf.config_scene("C2")
    W, H = 1920, 1080
    fp = cf.frame_params(W, H, max_bounce=1)
    ro = cf.rand_origins(1024)
    out = []
    for budget in (1 << 40, 48 * W * H):
        r = Renderer(0)
        try:
            r.set_scene_soa(sd.soa, sd.nodes)
            r.set_env(env_maps[0], env_maps[1])
            r.resize(W, H)
            r.set_max_paths(budget)
            r.render(fp, ro)
            out.append(r.read_accum())
        finally:
            r.close()
    assert bit_mismatch(out[0], out[1])[0] == 0.0


@pytest.mark.parametrize("name", ["C3", "C4"])
def test_longest_first_work_order_keeps_the_image(gpu_renderer, env_maps, name):
    """rt_order_work reorders the pixel list by 64-pixel blocks of descending probe cost: every
    later frame still equals the oracle bit for bit, one and several frames per call, and the
    probe leaves LoopNum and the accumulation as they were."""
    sd = cf.config_scene(name)
    W, H = 96, 72
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 3)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*env_maps)
    r.resize(W, H)
    r.order_work(fp, cf.rand_origins(1))
    assert r.loop_num == 0
    r.reset_stats()  # (the probe frame's rays are counted too)
    r.render(fp, ro[:1])
    st = r.render(fp, ro[1:])
    img = r.read_accum()
    assert bit_mismatch(img, ref)[0] == 0.0
    assert st["rays"] == cnt["rays"]


@pytest.mark.parametrize("name,depth", [("C3", 2), ("C4", 3)])
def test_pipelined_calls_match_oracle(gpu_renderer, env_maps, name, depth):
    """rt_set_pipeline: one-frame calls and one-batch calls in flight together (alternating
    streams, path-state sets, camera and frame tables), a camera that moves between calls, a host
    read and a two-batch (unpipelined) call in between: the image equals the oracle bit for bit at
    every read, and so does the ray count."""
    sd = cf.config_scene(name)
    W, H = 96, 72
    fps = [cf.frame_params(W, H, position=(0.05 * k, 0.1 * (k % 3), 7.0 - 0.2 * k)) for k in range(10)]
    ro = cf.rand_origins(10)
    # calls: three one-frame, one of 3 frames (two batches of at most 2), one of 2 frames (one
    # batch: pipelined), two one-frame; each call's frames use its first frame's camera
    calls = [(0, 1), (1, 1), (2, 1), (3, 3), (6, 2), (8, 1), (9, 1)]
    frames = [cf.oracle_frame_params(fps[k0], k + 1, ro[k]) for k0, n in calls for k in range(k0, k0 + n)]
    ref3, _ = oracle_render(sd, env_maps, W, H, frames[:3])
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*env_maps)
    r.resize(W, H)
    r.set_max_paths(2 * W * H)  # at most 2 frames per batch
    r.set_pipeline(depth)
    r.order_work(fps[0], cf.rand_origins(1))
    r.reset_stats()
    for i, (k0, n) in enumerate(calls):
        r.render_async(fps[k0], ro[k0:k0 + n])
        if i == 2:
            assert bit_mismatch(r.read_accum(), ref3)[0] == 0.0
    st = r.stats()
    assert r.loop_num == 10
    assert bit_mismatch(r.read_accum(), ref)[0] == 0.0
    assert st["rays"] == cnt["rays"]
    r.set_pipeline(1)
    r.set_max_paths(0)


@pytest.mark.parametrize("n,cap", [(11, 4), (9, 4), (6, 2)])
def test_batches_of_one_call_match_oracle(gpu_renderer, env_maps, n, cap):
    """A call of more frames than the path budget holds runs as several batches of frame groups
    (a last batch of one frame splits by pixels): the image and the ray count equal the oracle's."""
    sd = cf.config_scene("C3")
    W, H = 80, 56
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, n)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*env_maps)
    r.resize(W, H)
    r.set_max_paths(cap * W * H)
    r.reset_stats()
    st = r.render(fp, ro)
    assert bit_mismatch(r.read_accum(), ref)[0] == 0.0
    assert st["rays"] == cnt["rays"]
    assert st["launches"] == (n + cap - 1) // cap
    r.set_max_paths(0)


def test_env_angle_changes_between_calls_match_oracle(gpu_renderer, env_maps):
    """envAngle (RT:630) per call: the NEE light table (SampleHdrLight) is rebuilt whenever a
    call's angle differs, including across pipelined one-frame calls; every frame equals the
    oracle's with that frame's angle, and the image and ray count match."""
    sd = cf.config_scene("C3")
    W, H = 96, 64
    # two tables (one per angle in use): rebuilt on the call's stream after the last call that read
    # the table; an angle still held by the other table is reused (0.1 after 0.0)
    angles = [0.0, 0.25, 0.25, -0.4, 0.1, 0.0, 0.1, 0.1, -0.4, 0.0]
    ro = cf.rand_origins(len(angles))
    fps = [cf.frame_params(W, H, env_angle=a) for a in angles]
    frames = [cf.oracle_frame_params(fps[k], k + 1, ro[k]) for k in range(len(angles))]
    ref, cnt = oracle_render(sd, env_maps, W, H, frames)
    r = gpu_renderer
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*env_maps)
    r.resize(W, H)
    r.set_pipeline(2)
    r.reset_stats()
    for k in range(len(angles)):
        r.render_async(fps[k], ro[k:k + 1])
    st = r.stats()
    assert bit_mismatch(r.read_accum(), ref)[0] == 0.0
    assert st["rays"] == cnt["rays"]
    r.set_pipeline(1)


@pytest.mark.parametrize("depth", [1, 2])
def test_thousands_of_calls_without_synchronize(gpu_renderer, env_maps, depth):
    """A front end that never calls rt_synchronize: more one-frame calls than the context keeps
    timing-event pairs for (kMaxPendingEvents = 4096, rt_render.hip fold_events), with the pixel-
    split groups (depth 1) or pipelined calls on alternating streams (depth 2), so the oldest
    pairs are folded while later ones, on other streams, are still running.  Every call succeeds,
    and the image and ray count equal one batched call of the same frames (itself bit-exact vs
    the oracle elsewhere)."""
    sd = cf.config_scene("C2")
    W, H = 16, 16
    n = 1100 if depth == 1 else 2100  # 4 / 2 trace-event pairs per call
    fp = cf.frame_params(W, H)
    ro = cf.rand_origins(n)
    r = gpu_renderer
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*env_maps)
    r.resize(W, H)
    r.reset_stats()
    st = r.render(fp, ro)
    ref = r.read_accum()
    r.resize(W, H)
    r.set_pipeline(depth)
    r.reset_stats()
    try:
        for k in range(n):
            r.render_async(fp, ro[k:k + 1])
        st2 = r.stats()
    finally:
        r.set_pipeline(1)
    assert r.loop_num == n
    assert bit_mismatch(r.read_accum(), ref)[0] == 0.0
    assert st2["rays"] == st["rays"]
    assert st2["launches"] == n
    # the traversal launches' busy union (folded in bounded memory: intervals of calls <= k-2 are
    # summed and dropped) lies within the calls' summed time and is not empty
    assert 0.0 < st2["trace_busy_ms"] <= st2["kernel_ms"] * 1.001, st2


def test_bench_operating_point_matches_oracle(gpu_renderer, env_maps):
    """bench.py's operating point, pinned against the oracle.  The bench renders
    C3 in 1024-frame calls at loopNum 1 .. 25,600 (5 warm-up + 20 timed steps), each call two
    launches of 512 frames (the path-state budget), each launch two frame groups of 256 frames
    traced by the bulk kernels (groups of 530 M slots, far above the finisher's limit).  Here the
    same shape at 48x27: one call of 1024 frames at loopNum 24,001 .. 25,024 (randOrigin from the
    same glibc sequence, Sobol indices loopNum + 1 up to 25,025, RT:616-620), a budget of 512
    frames (two launches), the finisher's slot limit at 1 (every group on the bulk kernels), over a
    host-written history as if 24,000 frames were accumulated (the blend weights {1/n, (n-1)/n}
    at n ~ 25 k, RT:1552).  Image bit for bit and the device ray count equal the oracle's."""
    sd = cf.config_scene("C3")
    W, H = 48, 27
    first, n = 24001, 1024
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, first, n, ro_offset=first - 1)
    hist = np.random.default_rng(5).uniform(0.0, 2.0, (H, W, 3)).astype(np.float32)
    ref, cnt = oracle_render(sd, env_maps, W, H, frames, accum=hist)
    r = gpu_renderer
    r.set_max_paths(512 * W * H)
    r.set_finish(2, 1)
    try:
        img, st = gpu_render(r, sd, env_maps, W, H, fp, ro, accum=hist, loop_num=first - 1)
    finally:
        r.set_max_paths(0)
        r.set_finish(2, 8 << 20)
    assert r.loop_num == first + n - 1
    assert st["launches"] == 2 and st["trace_launches"] == 2 * 2 * 9, st  # batches x groups x passes
    assert st["finish_steps"] == 0 and st["samples"] == W * H * n
    assert st["rays"] == cnt["rays"], (st, cnt)
    assert bit_mismatch(img, ref)[0] == 0.0


def test_stats_get_writes_the_abi3_struct_only(gpu_renderer, env_maps):
    """ABI 5: rt_stats_get (and rt_render's stats argument) write the 104 bytes of the ABI-3 rt_stats
    a binding of that header allocated, never the fields added since; rt_stats_get_sized with the
    full size returns those."""
    import ctypes as C
    from rtamd.renderer import RtStats
    sd = cf.config_scene("C2")
    W, H = 32, 32
    fp = cf.frame_params(W, H)
    ro, _ = frames_for(fp, 1, 2)
    gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    L, h = gpu_renderer._L, gpu_renderer._h
    buf = (C.c_uint8 * 256)(*([0xAB] * 256))
    assert L.rt_stats_get(h, C.cast(buf, C.POINTER(RtStats))) == 0
    assert all(b == 0xAB for b in bytes(buf)[104:]), "rt_stats_get wrote past the ABI-3 struct"
    full = gpu_renderer.stats()
    assert int.from_bytes(bytes(buf)[0:8], "little") == full["rays"] > 0
    assert full["pass0_steps"] > 0 and full["trace_busy_ms"] > 0.0
    buf2 = (C.c_uint8 * 256)(*([0xAB] * 256))
    p = C.cast(buf2, C.POINTER(RtStats))
    assert L.rt_render(h, C.byref(fp.to_c()), ro.ctypes.data_as(C.POINTER(C.c_float)), 1, p) == 0
    assert all(b == 0xAB for b in bytes(buf2)[104:]), "rt_render wrote past the ABI-3 struct"
