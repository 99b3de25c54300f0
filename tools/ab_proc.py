#!/usr/bin/env python3
"""Process-per-measurement A/B timing (development aid): every measurement is a fresh process
with one context (as in bench.py), the variants interleaved over rounds, so neither box-to-box
noise nor the in-process position effects of tools/ab_inproc.py (hardware-queue sharing between
contexts) bias a comparison.

    python tools/ab_proc.py --rounds 3 base=default x=path/to/librtamd_x.so y=default:RT_GROUPS=3
    python tools/ab_proc.py --one path-or-default [--frames 512]     (one measurement, internal)
"""
import argparse
import json
import os
import statistics
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("variants", nargs="*")
ap.add_argument("--config", default="C3")
ap.add_argument("--frames", type=int, default=512)
ap.add_argument("--reps", type=int, default=2, help="timed render calls per measurement")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--one", default=None)
ap.add_argument("--whole", action="store_true", help="path budget = frames x pixels (bench.py's setting)")
a = ap.parse_args()

if a.one is not None:
    from rtamd import configs as cf
    from rtamd.renderer import Renderer
    cfg = cf.CONFIGS[a.config]
    W, H = cfg.width, cfg.height
    sd = cf.config_scene(a.config)
    r = Renderer(0, lib_path=None if a.one == "default" else a.one)
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*cf.load_env())
    r.resize(W, H)
    if a.whole:
        r.set_max_paths(a.frames * W * H)
    fp = cf.frame_params(W, H)
    ro = cf.rand_origins(a.frames)
    if os.environ.get("RT_AB_ORDER"):  # rt_order_work from one probe frame before timing
        r.order_work(fp, ro[:1])
    r.render(fp, ro)
    r.reset_stats()
    r.synchronize()
    t = time.perf_counter()
    for _ in range(a.reps):
        r.render_async(fp, ro)
    r.synchronize()
    dt = time.perf_counter() - t
    st = r.stats()
    print(json.dumps({"mrays": st["rays"] / dt / 1e6, "ms_per_frame": dt * 1e3 / (a.reps * a.frames)}))
    sys.exit(0)

specs = []
for v in a.variants:
    name, rest = v.split("=", 1)
    path, _, envs = rest.partition(":")
    env = dict(e.split("=", 1) for e in envs.split(",") if e)
    specs.append((name, path if path == "default" else str(Path(path).resolve()), env))
res = {n: [] for n, _, _ in specs}
for rnd in range(a.rounds):
    for name, path, env in specs:
        p = subprocess.run([sys.executable, __file__, "--one", path, "--config", a.config, "--frames", str(a.frames),
                            "--reps", str(a.reps)] + (["--whole"] if a.whole else []), env={**os.environ, **env}, capture_output=True, text=True,
                           timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:], flush=True)
            sys.exit(p.returncode)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        res[name].append(d["mrays"])
        print(f"round {rnd} {name:12s} {d['mrays']:8.1f} Mrays/s  {d['ms_per_frame']:.3f} ms/frame", flush=True)
base = statistics.median(res[specs[0][0]])
print("median Mrays/s (vs first):")
for name, _, _ in specs:
    m = statistics.median(res[name])
    print(f"  {name:12s} {m:8.1f}  {m / base - 1:+.2%}  spread {min(res[name]):.0f}-{max(res[name]):.0f}")
