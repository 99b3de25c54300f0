"""Parity at the BASELINE.json configurations' full sizes.

* Whole frames of C2 (1280x720), C3 / C4 (1920x1080) and C5 (3840x2160) rendered by the HIP
  path equal the oracle bit for bit (every pixel, every channel), and the device ray count
  equals the oracle's hitBVH count.  The oracle runs on at most 16 host threads (a 1080p frame
  of C3 takes ~0.5 s there).
* Size-independent properties at 1080p, where the oracle would take too long for many frames:
  - 8-rank tile split + device assembly == the single-rank render (pixels are independent);
  - frames in flight: one call of 32 frames == 32 calls of one frame (blend in frame order);
  - progressive history: 16 + 16 frames across two calls == 32 frames in one call.
"""
import os

import numpy as np
import pytest

from helpers import bit_mismatch, frames_for, gpu_render
from rtamd import configs as cf

pytestmark = pytest.mark.gpu


def _threads() -> int:
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return max(1, min(16, os.cpu_count() or 1))


def _oracle(sd, env, W, H, frames):
    import oracle as orc
    scene = orc.OracleScene(sd.tri_enc, sd.node_enc, env[0], env[1])
    return orc.render(scene, frames, W, H, threads=_threads())


@pytest.mark.parametrize("name,n_frames", [("C2", 2), ("C3", 2), ("C4", 1), ("C5", 1)])
def test_full_frame_matches_oracle(gpu_renderer, env_maps, name, n_frames):
    cfg = cf.CONFIGS[name]
    W, H = cfg.width, cfg.height
    sd = cf.config_scene(name)
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, n_frames)
    ref, cnt = _oracle(sd, env_maps, W, H, frames)
    img, st = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    frac, diff = bit_mismatch(img, ref)
    assert frac == 0.0, f"{name} {W}x{H}: {int(diff.sum())} pixels differ"
    assert st["rays"] == cnt["rays"]
    assert st["samples"] == W * H * n_frames


def test_full_size_eight_rank_tiles_equal_single_rank(gpu_renderer, env_maps):
    import torch
    from rtamd.renderer import Renderer
    sd = cf.config_scene("C3")
    W, H, world = 1920, 1080, 8
    fp = cf.frame_params(W, H)
    ro, _ = frames_for(fp, 1, 4)
    single, st1 = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro)
    parts, rays = [], 0
    ctx = Renderer(0)
    try:
        for rank in range(world):
            _, st = gpu_render(ctx, sd, env_maps, W, H, fp, ro, rank=rank, world=world)
            rays += st["rays"]
            info = ctx.accum_device()
            buf = torch.empty(info["bytes"] // 4, dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            ctx.copy_accum_device(buf.data_ptr(), info["bytes"])
            ctx.synchronize()
            parts.append(buf)
        gathered = torch.cat(parts)
        frame = torch.empty(H * W * 3, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        ctx.assemble_frame(gathered.data_ptr(), world, frame.data_ptr())
        ctx.synchronize()
        torch.cuda.synchronize()
        img = frame.cpu().numpy().reshape(H, W, 3)
    finally:
        ctx.close()
    assert bit_mismatch(img, single)[0] == 0.0
    assert rays == st1["rays"]


def test_full_size_frames_in_flight_and_history(gpu_renderer, env_maps):
    sd = cf.config_scene("C3")
    W, H, n = 1920, 1080, 32
    fp = cf.frame_params(W, H)
    ro = cf.rand_origins(n)
    r = gpu_renderer
    all_at_once, st_all = gpu_render(r, sd, env_maps, W, H, fp, ro)
    # one frame per call
    r.clear_accum()
    r.reset()
    r.reset_stats()
    for k in range(n):
        r.render_async(fp, ro[k:k + 1])
    one_by_one = r.read_accum()
    st_one = r.stats()
    # one frame per call, pipelined (rt_set_pipeline: calls in flight together)
    r.clear_accum()
    r.reset()
    r.set_pipeline(2)
    for k in range(n):
        r.render_async(fp, ro[k:k + 1])
    pipelined = r.read_accum()
    r.set_pipeline(1)
    # two calls of 16 frames (progressive history carried in the accumulation buffer)
    r.clear_accum()
    r.reset()
    r.render_async(fp, ro[:16])
    r.render(fp, ro[16:])
    halves = r.read_accum()
    assert r.loop_num == n
    assert bit_mismatch(one_by_one, all_at_once)[0] == 0.0
    assert bit_mismatch(pipelined, all_at_once)[0] == 0.0
    assert bit_mismatch(halves, all_at_once)[0] == 0.0
    assert st_one["rays"] == st_all["rays"]
    assert np.isfinite(all_at_once).mean() > 0.99
