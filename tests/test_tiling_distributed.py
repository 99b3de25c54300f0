"""Multi-GPU sharding path on CPU: world_size-2 gloo processes render their pixel tiles
(with the oracle standing in for each rank's GPU), gather them to rank 0 exactly as bench.py
does over RCCL, and the un-permuted frame equals the single-process render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT
from rtamd import tiling

W, H, TILE = 40, 24, 8


def _render_rank(rank, world, owner=None, costs_only=False):
    import sys
    sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as orc
    from rtamd import configs as cf
    sd = cf.config_scene("C2")
    env = cf.load_env()
    fp = cf.frame_params(W, H)
    ro = cf.rand_origins(1)
    sc = orc.OracleScene(sd.tri_enc, sd.node_enc, env[0], env[1])
    frames = [cf.oracle_frame_params(fp, 1, ro[0])]
    mlt = tiling.max_local_tiles(W, H, TILE, TILE, world, owner)
    buf = np.zeros((mlt, TILE, TILE, 4), np.float32)
    costs = {}
    for lt, t in enumerate(tiling.local_tiles(W, H, TILE, TILE, rank, world, owner)):
        x0, y0, w, h = tiling.tile_rect(t, W, H, TILE, TILE)
        img, cnt = orc.render(sc, frames, W, H, x0=x0, y0=y0, w=w, h=h, threads=1)
        buf[lt, :h, :w, :3] = img
        costs[t] = int(cnt["tri_tests"] + cnt["internal_pops"] + 16 * cnt["rays"])
    return costs if costs_only else buf


def _worker(rank, world, port, out_path, balanced=False):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    owner = None
    if balanced:
        # bench.py's flow: each rank measures its default tiles' costs (the oracle's visit counts
        # stand in for rt_tile_costs), all ranks exchange them and derive the same owner map
        mine = _render_rank(rank, world, costs_only=True)
        allc = [None] * world
        dist.all_gather_object(allc, mine)
        costs = np.zeros(len(tiling.modulo_owners(W, H, TILE, TILE, world)), np.int64)
        for d in allc:
            for t, c in d.items():
                costs[t] = c
        owner = tiling.balance(costs, world)
    local = torch.from_numpy(_render_rank(rank, world, owner))
    parts = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, gather_list=parts, dst=0)
    if rank == 0:
        g = torch.stack(parts).numpy()
        frame = tiling.assemble(g, W, H, TILE, TILE, world, owner)
        np.save(out_path, frame[..., :3])
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("balanced", [False, True], ids=["modulo", "cost-balanced"])
@pytest.mark.parametrize("world", [2])
def test_two_rank_gather_equals_single_render(tmp_path, world, balanced):
    out = tmp_path / "frame.npy"
    mp.spawn(_worker, args=(world, _free_port(), str(out), balanced), nprocs=world, join=True)
    frame = np.load(out)
    single = tiling.assemble(_render_rank(0, 1)[None], W, H, TILE, TILE, 1)[..., :3]
    assert np.array_equal(frame.view(np.uint32), single.view(np.uint32))


def test_tile_ownership_partitions_the_frame():
    for world in (1, 2, 3, 8):
        seen = np.zeros((H, W), np.int32)
        for r in range(world):
            for t in tiling.local_tiles(W, H, TILE, TILE, r, world):
                x0, y0, w, h = tiling.tile_rect(t, W, H, TILE, TILE)
                seen[y0:y0 + h, x0:x0 + w] += 1
        assert np.all(seen == 1)


def test_balance_is_a_deterministic_even_partition():
    rng = np.random.default_rng(0)
    costs = (rng.pareto(1.5, size=2040) * 1000).astype(np.int64)
    for world in (1, 2, 4, 8):
        o1 = tiling.balance(costs, world)
        assert np.array_equal(o1, tiling.balance(costs.copy(), world))
        loads = np.bincount(o1, weights=costs, minlength=world)
        assert loads.max() - loads.mean() <= costs.max()
        mod = np.bincount(tiling.modulo_owners(1920, 1088, 32, 32, world), weights=costs, minlength=world)
        assert loads.max() <= mod.max()
        seen = np.zeros((1088 // 32) * 60, np.int32)
        for r in range(world):
            seen[tiling.local_tiles(1920, 1088, 32, 32, r, world, o1)] += 1
        assert np.all(seen == 1)
