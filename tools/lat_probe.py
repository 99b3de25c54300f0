#!/usr/bin/env python3
"""Single-frame latency of one context under the conditions bench.py measures it in (development
aid): default path slots, then bench's rt_set_max_paths (1024 frames' slots), then after a
bulk render (1024-frame calls), each as the median of synchronised one-frame calls."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

TORCH_FIRST = "--torch-first" in sys.argv
if TORCH_FIRST:  # as bench.py: torch's stream made first and handed to the renderer
    import torch
    torch.cuda.set_device(0)
    tstream = torch.cuda.Stream()
    torch.cuda.set_stream(tstream)
cfg = cf.CONFIGS["C3"]
W, H = cfg.width, cfg.height
sd = cf.config_scene("C3")
r = Renderer(0)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*cf.load_env())
if TORCH_FIRST:
    r.set_stream(tstream.cuda_stream)
r.resize(W, H)
fp = cf.frame_params(W, H)
OFF = int(sys.argv[sys.argv.index("--ro-offset") + 1]) if "--ro-offset" in sys.argv else 0
ro = cf.rand_origins(OFF + 2200)[OFF:]


PF = int(sys.argv[sys.argv.index("--probe-frames") + 1]) if "--probe-frames" in sys.argv else 1


def lat(tag, n=24):
    r.order_work(fp, ro[:PF])
    for k in range(4):
        r.render_async(fp, ro[k:k + 1])
    r.synchronize()
    t = time.perf_counter()
    for k in range(n):
        r.render_async(fp, ro[k:k + 1])
    r.synchronize()
    b2b = (time.perf_counter() - t) * 1e3 / n
    s = []
    for k in range(n):
        t = time.perf_counter()
        r.render_async(fp, ro[k:k + 1])
        r.synchronize()
        s.append(time.perf_counter() - t)
    print(f"{tag:40s} b2b {b2b:.3f} ms  sync median {np.median(s) * 1e3:.3f} ms", flush=True)


lat("default slots")
r.set_max_paths(1024 * W * H)
lat("max paths 1024 frames")
for k in range(3):
    r.render_async(fp, ro[100:100 + 1024])
r.synchronize()
lat("after 3 bulk 1024-frame calls")
time.sleep(2.0)
lat("after 2 s idle")
r.set_pipeline(2)
lat("pipeline depth 2")
r.set_pipeline(1)
lat("pipeline depth 1 after depth 2")
if TORCH_FIRST:
    r.set_stream(None)
    lat("own stream again")
