#!/usr/bin/env python3
"""Per-rank scaling estimate on one GPU: rank 0's tile share of an N-rank run (bench.py's
tiling and path budget), timed alone for N = 1, 2, 4, 8.  Strong-scaling efficiency of the
render part = t(1) / (N * t(N)) (the frame-end gather is not included)."""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=512)
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--worlds", default="1,2,4,8")
a = ap.parse_args()
sd = cf.config_scene("C3")
env = cf.load_env()
W, H = 1920, 1080
fp = cf.frame_params(W, H)
ro = cf.rand_origins(a.frames)
t1 = None
for world in [int(x) for x in a.worlds.split(",")]:
    r = Renderer(0)
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*env)
    r.resize(W, H, tile=32, rank=0, world=world)
    ad = r.accum_device()
    r.set_max_paths(a.frames * ad["local_tiles"] * 32 * 32)
    r.render(fp, ro)
    r.reset_stats()
    r.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        r.render_async(fp, ro)
    r.synchronize()
    dt = (time.perf_counter() - t) / a.reps
    st = r.stats()
    t1 = dt if t1 is None else t1
    print(f"world {world}: rank-0 step {dt * 1e3:.1f} ms, {st['rays'] / a.reps / dt / 1e6:.0f} Mrays/s per rank, "
          f"efficiency vs N=1 {t1 / (world * dt):.3f}", flush=True)
    r.close()
