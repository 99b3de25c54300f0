#!/usr/bin/env python3
"""In-process A/B timing of library builds and runtime settings (development aid).

Every variant is `name=path/to/librtamd_x.so` or `name=default`, optionally followed by
`:ENV=value,ENV2=value` (read by the library at rt_create / rt_set_scene).  The variants are
timed in interleaved rounds on the bench workload (C3 1080p, `--frames` per render call) with one
context per variant created up front (RT_MAX_SLOTS defaults to 160 Mi here so several contexts fit
in HBM: re-creating 69-GB contexts back to back left freed memory unreclaimed and later
contexts ran many times slower), so box-to-box noise cancels and drift shows up as spread.

    python tools/ab_inproc.py --rounds 5 a=default b=opengl-ray-tracing-framework_amd/lib/exp/librtamd_x.so
"""
import argparse
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="+")
ap.add_argument("--config", default="C3")
ap.add_argument("--frames", type=int, default=512)
ap.add_argument("--rounds", type=int, default=5)
a = ap.parse_args()

specs = []
for v in a.variants:
    name, rest = v.split("=", 1)
    path, _, envs = rest.partition(":")
    env = dict(e.split("=", 1) for e in envs.split(",") if e)
    specs.append((name, None if path == "default" else str(Path(path).resolve()), env))

cfg = cf.CONFIGS[a.config]
W, H = cfg.width, cfg.height
sd = cf.config_scene(a.config)
env_maps = cf.load_env()
fp = cf.frame_params(W, H)
ro = cf.rand_origins(a.frames)
results = {n: [] for n, _, _ in specs}
ctx = {}
for name, path, env in specs:
    env = {"RT_MAX_SLOTS": str(160 << 20), **env}
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        r = Renderer(0, lib_path=path)
        r.set_scene_soa(sd.soa, sd.nodes)
        r.set_env(*env_maps)
        r.resize(W, H)
        r.render(fp, ro)  # full-size allocations once (a smaller first call re-allocates later), code objects
        r.synchronize()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ctx[name] = r
for rnd in range(a.rounds):
    for name, _, _ in specs:
        r = ctx[name]
        r.reset()
        r.reset_stats()
        r.synchronize()
        t = time.perf_counter()
        r.render_async(fp, ro)
        r.synchronize()
        dt = time.perf_counter() - t
        st = r.stats()
        results[name].append(st["rays"] / dt / 1e6)
        print(f"round {rnd} {name:12s} {results[name][-1]:8.1f} Mrays/s  {dt * 1e3 / a.frames:.3f} ms/frame", flush=True)
base = statistics.median(results[specs[0][0]])
print("median Mrays/s (vs first):")
for name, _, _ in specs:
    m = statistics.median(results[name])
    print(f"  {name:12s} {m:8.1f}  {m / base - 1:+.2%}  spread {min(results[name]):.0f}-{max(results[name]):.0f}")
