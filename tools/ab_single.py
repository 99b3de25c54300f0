#!/usr/bin/env python3
"""Process-per-measurement A/B timing of single-frame render calls (the reference's own usage:
one frame per rt_render, main.cpp:175-200), variants interleaved over rounds (development aid).

    python tools/ab_single.py --rounds 3 base=default x=path/to/librtamd_x.so y=default:RT_FINISH_PASS=0
    python tools/ab_single.py --one path-or-default          (one measurement, internal)

Prints per variant the median ms per back-to-back call and per synchronised call.
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
ap.add_argument("--calls", type=int, default=48)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--one", default=None)
a = ap.parse_args()

if a.one is not None:
    import numpy as np

    from rtamd import configs as cf
    from rtamd.renderer import Renderer
    cfg = cf.CONFIGS[a.config]
    W, H = cfg.width, cfg.height
    sd = cf.config_scene(a.config)
    r = Renderer(0, lib_path=None if a.one == "default" else a.one)
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*cf.load_env())
    r.resize(W, H)
    fp = cf.frame_params(W, H)
    ro = cf.rand_origins(8 + a.calls + 16)
    if os.environ.get("RT_AB_PIPE"):  # rt_set_pipeline depth (frames in flight across calls)
        r.set_pipeline(int(os.environ["RT_AB_PIPE"]))
    if os.environ.get("RT_AB_ORDER"):  # rt_order_work from one probe frame before timing
        r.order_work(fp, ro[:1])
    for k in range(8):
        r.render_async(fp, ro[k:k + 1])
    r.synchronize()
    t = time.perf_counter()
    for k in range(a.calls):
        r.render_async(fp, ro[8 + k:9 + k])
    r.synchronize()
    b2b = (time.perf_counter() - t) * 1e3 / a.calls
    lat = []
    for k in range(16):
        t = time.perf_counter()
        r.render(fp, ro[8 + a.calls + k:9 + a.calls + k])
        lat.append((time.perf_counter() - t) * 1e3)
    print(json.dumps({"b2b_ms": b2b, "lat_ms": float(np.median(lat))}))
    sys.exit(0)

specs = []
for v in a.variants:
    name, rest = v.split("=", 1)
    path, _, envs = rest.partition(":")
    env = dict(e.split("=", 1) for e in envs.split(",") if e)
    specs.append((name, path if path == "default" else str(Path(path).resolve()), env))
res = {n: ([], []) for n, _, _ in specs}
for rnd in range(a.rounds):
    for name, path, env in specs:
        p = subprocess.run([sys.executable, __file__, "--one", path, "--config", a.config, "--calls", str(a.calls)],
                           env={**os.environ, **env}, capture_output=True, text=True, timeout=300)
        if p.returncode != 0:
            print(p.stderr[-2000:], flush=True)
            sys.exit(p.returncode)
        d = json.loads(p.stdout.strip().splitlines()[-1])
        res[name][0].append(d["b2b_ms"])
        res[name][1].append(d["lat_ms"])
        print(f"round {rnd} {name:12s} {d['b2b_ms']:7.3f} ms/call back-to-back  {d['lat_ms']:7.3f} ms synchronised", flush=True)
print("median ms per single-frame call (back-to-back / synchronised):")
base = statistics.median(res[specs[0][0]][0])
for name, _, _ in specs:
    b, l = statistics.median(res[name][0]), statistics.median(res[name][1])
    print(f"  {name:12s} {b:7.3f} ({b / base - 1:+.1%})  {l:7.3f}   spread {min(res[name][0]):.3f}-{max(res[name][0]):.3f}")
