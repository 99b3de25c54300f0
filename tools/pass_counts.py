#!/usr/bin/env python3
"""Per-pass ray counts and durations of one-frame render calls (development aid, RT_DEV library).

    RT_DEBUG_PASSES=1 RT_FINISH_PASS=99 python3 tools/pass_counts.py [--config C3] [--frames 1]

Loads lib/librtamd_dev.so, renders warm-up frames, then one call of --frames frames with the
per-pass report (stderr) of rt_render.hip's RT_DEBUG_PASSES."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import Renderer, dev_lib_path  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--frames", type=int, default=1)
ap.add_argument("--count", action="store_true", help="RT_FLAG_COUNT_VISITS: steps-per-ray histograms per pass")
ap.add_argument("--lib", default=None, help="library (default lib/librtamd_dev.so)")
ap.add_argument("--warm", type=int, default=0, help="one-frame calls before the measured one (timelines)")
ap.add_argument("--order", action="store_true", help="rt_order_work from one probe frame first (as bench.py does)")
ap.add_argument("--max-paths", type=int, default=0, help="rt_set_max_paths (0: default budget)")
a = ap.parse_args()
cfg = cf.CONFIGS[a.config]
W, H = cfg.width, cfg.height
sd = cf.config_scene(a.config)
r = Renderer(0, lib_path=a.lib or dev_lib_path())
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*cf.load_env())
r.resize(W, H)
if a.max_paths:
    r.set_max_paths(a.max_paths)
from rtamd.renderer import RT_FLAG_COUNT_VISITS  # noqa: E402
fp = cf.frame_params(W, H, flags=RT_FLAG_COUNT_VISITS if a.count else 0)
ro = cf.rand_origins(max(8, a.frames))
if a.order:
    r.order_work(cf.frame_params(W, H), ro[:1])
for k in range(a.warm):
    r.render(cf.frame_params(W, H), ro[k % 8:k % 8 + 1])
print("---- measured call", file=sys.stderr, flush=True)
st = r.render(fp, ro[:a.frames])
print(st, flush=True)
