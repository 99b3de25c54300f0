#!/usr/bin/env python3
"""Single-frame latency after repeated rt_order_work probes (development aid): per probe, the
median / min / max of 24 synchronised one-frame calls, to see how much the work order chosen from
the probe frames moves the latency."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

PF = int(sys.argv[1]) if len(sys.argv) > 1 else 1
cfg = cf.CONFIGS["C3"]
W, H = cfg.width, cfg.height
sd = cf.config_scene("C3")
r = Renderer(0)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*cf.load_env())
r.resize(W, H)
fp = cf.frame_params(W, H)
ro = cf.rand_origins(40000)
OFF = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
NP = int(sys.argv[3]) if len(sys.argv) > 3 else 8


def measure(base):
    s = []
    for k in range(32):
        t = time.perf_counter()
        r.render_async(fp, ro[base + k:base + k + 1])
        r.synchronize()
        s.append((time.perf_counter() - t) * 1e3)
    return np.median(s)


for probe in range(NP):
    r.order_work(fp, ro[OFF + probe * PF:OFF + (probe + 1) * PF])
    r.render(fp, ro[:1])
    a, b = measure(100), measure(200)
    print(f"probe {probe} ({PF} frames at {OFF + probe * PF}): sync median {a:.3f} / again {b:.3f}", flush=True)
