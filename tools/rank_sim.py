#!/usr/bin/env python3
"""Per-rank balance of the N-rank bench on one GPU: EVERY rank's tile share of an N-rank run
(bench.py's tiling, frames per step and path budget) rendered alone, for N = 1, 2, 4, 8.

The bench's value at N ranks is rays of all ranks / the slowest rank's time, so the render part's
strong-scaling efficiency is t(1) / (N * max_r t_r(N)); the imbalance max/mean says how much of
the loss is the tile assignment (the frame-end gather is not included).  Prints one JSON line
per N and, with --out, writes them all to a file.

    python tools/rank_sim.py [--frames 1024] [--reps 1] [--worlds 1,2,4,8]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
from rtamd import configs as cf  # noqa: E402
from rtamd import tiling  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--frames", type=int, default=1024)
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--worlds", default="1,2,4,8")
ap.add_argument("--tile", type=int, default=32)
ap.add_argument("--out", default=None)
ap.add_argument("--probe-frames", type=int, default=1, help="frames of the tile-cost probe (bench.py: 1)")
ap.add_argument("--pipeline", type=int, default=1, help="rt_set_pipeline depth (calls in flight together)")
ap.add_argument("--calls", type=int, default=1, help="render calls per step (the step's frames split evenly)")
ap.add_argument("--assign", default="both", choices=["modulo", "balanced", "both"],
                help="tile owner map: interleaved t %% N, bench.py's cost-balanced map, or both")
a = ap.parse_args()
cfg = cf.CONFIGS[a.config]
sd = cf.config_scene(a.config)
env = cf.load_env()
W, H = cfg.width, cfg.height
fp = cf.frame_params(W, H)
ro = cf.rand_origins(a.frames + a.probe_frames)
r = Renderer(0)
r.set_pipeline(a.pipeline)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*env)
lines = []
# full-frame tile costs (what bench.py's ranks assemble from their shares with an all_reduce)
r.resize(W, H, tile=a.tile)
costs = r.tile_costs(fp, ro[-a.probe_frames:])
t1 = None
modes = ["modulo", "balanced"] if a.assign == "both" else [a.assign]
for world, mode in [(int(x), m) for x in a.worlds.split(",") for m in modes]:
    if world == 1 and mode == "balanced" and "modulo" in modes:
        continue  # (one rank owns every tile either way)
    owner = tiling.balance(costs, world) if mode == "balanced" and world > 1 else None
    times, rays = [], []
    for rank in range(world):
        r.resize(W, H, tile=a.tile, rank=rank, world=world)
        if owner is not None:
            r.set_tile_owners(owner)
        ad = r.accum_device()
        r.set_max_paths(a.frames * ad["local_tiles"] * a.tile * a.tile)
        per = a.frames // a.calls
        for c in range(a.calls):                  # warm: path-state allocation, first launches
            r.render_async(fp, ro[1 + c * per:1 + (c + 1) * per])
        r.synchronize()
        r.reset_stats()
        t = time.perf_counter()
        for _ in range(a.reps):
            for c in range(a.calls):
                r.render_async(fp, ro[1 + c * per:1 + (c + 1) * per])
        r.synchronize()
        times.append((time.perf_counter() - t) / a.reps)
        rays.append(r.stats()["rays"] / a.reps)
    tmax, tmean = max(times), sum(times) / len(times)
    t1 = tmax if t1 is None else t1
    d = {"config": a.config, "world": world, "assign": mode, "frames": a.frames, "pipeline": a.pipeline, "calls": a.calls, "rank_ms": [round(x * 1e3, 1) for x in times],
         "max_ms": round(tmax * 1e3, 1), "mean_ms": round(tmean * 1e3, 1), "imbalance": round(tmax / tmean, 4),
         "mrays_per_s_job": round(sum(rays) / tmax / 1e6, 1), "efficiency_vs_n1": round(t1 / (world * tmax), 4)}
    lines.append(d)
    print(json.dumps(d), flush=True)
r.close()
if a.out:
    Path(a.out).write_text("\n".join(json.dumps(x) for x in lines) + "\n")
