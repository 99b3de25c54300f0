#!/usr/bin/env python3
"""Single-frame latency before and after sustained bulk load (development aid): synchronised
one-frame calls, then ~25 s of 1024-frame calls (the bench's timed region), then the same
single-frame measurement right after and after idle pauses."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

cfg = cf.CONFIGS["C3"]
W, H = cfg.width, cfg.height
sd = cf.config_scene("C3")
r = Renderer(0)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*cf.load_env())
r.resize(W, H)
r.set_max_paths(1024 * W * H)
fp = cf.frame_params(W, H)
ro = cf.rand_origins(4000)


def lat(tag, n=64):
    s = []
    for k in range(n):
        t = time.perf_counter()
        r.render_async(fp, ro[100 + k:101 + k])
        r.synchronize()
        s.append((time.perf_counter() - t) * 1e3)
    print(f"{tag:32s} sync median {np.median(s):.3f} ms (min {min(s):.3f})", flush=True)


r.order_work(fp, ro[:1])
r.render(fp, ro[:1])
lat("cold")
t = time.perf_counter()
n = 0
while time.perf_counter() - t < 25.0:
    r.render(fp, ro[1000:2024])
    n += 1
print(f"bulk: {n} x 1024 frames in {time.perf_counter() - t:.1f} s", flush=True)
lat("right after bulk")
time.sleep(3.0)
lat("after 3 s idle")
time.sleep(10.0)
lat("after 13 s idle")
