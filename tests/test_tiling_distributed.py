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


def _render_rank(rank, world):
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
    mlt = tiling.max_local_tiles(W, H, TILE, TILE, world)
    buf = np.zeros((mlt, TILE, TILE, 4), np.float32)
    for lt, t in enumerate(tiling.local_tiles(W, H, TILE, TILE, rank, world)):
        x0, y0, w, h = tiling.tile_rect(t, W, H, TILE, TILE)
        img, _ = orc.render(sc, frames, W, H, x0=x0, y0=y0, w=w, h=h, threads=1)
        buf[lt, :h, :w, :3] = img
    return buf


def _worker(rank, world, port, out_path):
    import torch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = torch.from_numpy(_render_rank(rank, world))
    parts = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
    dist.gather(local, gather_list=parts, dst=0)
    if rank == 0:
        g = torch.stack(parts).numpy()
        frame = tiling.assemble(g, W, H, TILE, TILE, world)
        np.save(out_path, frame[..., :3])
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2])
def test_two_rank_gather_equals_single_render(tmp_path, world):
    out = tmp_path / "frame.npy"
    mp.spawn(_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
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
