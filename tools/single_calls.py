#!/usr/bin/env python3
"""Synchronised one-frame render calls of C3 1080p as bench.py's latency leg makes them (work order
from one probe frame, then N calls each followed by rt_synchronize) — a workload to run under
`rocprofv3 --kernel-trace` for tools/single_timeline.py (development aid).

    python3 tools/single_calls.py [--calls 8] [--config C3]
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--calls", type=int, default=8)
ap.add_argument("--config", default="C3")
a = ap.parse_args()
cfg = cf.CONFIGS[a.config]
W, H = cfg.width, cfg.height
sd = cf.config_scene(a.config)
r = Renderer(0)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*cf.load_env())
r.resize(W, H)
fp = cf.frame_params(W, H)
ro = cf.rand_origins(a.calls + 8)
r.order_work(fp, ro[:1])
for k in range(4):
    r.render_async(fp, ro[k:k + 1])
    r.synchronize()
lat = []
for k in range(a.calls):
    t = time.perf_counter()
    r.render_async(fp, ro[4 + k:5 + k])
    r.synchronize()
    lat.append(time.perf_counter() - t)
print(f"{a.config} one-frame calls, synchronised: median {np.median(lat) * 1e3:.3f} ms "
      f"(min {min(lat) * 1e3:.3f}, max {max(lat) * 1e3:.3f})", flush=True)
