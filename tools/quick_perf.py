#!/usr/bin/env python3
"""Quick GPU timing of one config (development aid; bench.py is the contract)."""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import RT_FLAG_COUNT_VISITS, Renderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--frames", type=int, default=4)
ap.add_argument("--per-launch", type=int, default=1)
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--max-bounce", type=int, default=8)
ap.add_argument("--flags", type=int, default=0)
ap.add_argument("--count-frames", type=int, default=1, help="frames of the visit-counting render")
a = ap.parse_args()
cfg = cf.CONFIGS[a.config]
W, H = a.width or cfg.width, a.height or cfg.height
t0 = time.time()
sd = cf.config_scene(a.config)
env = cf.load_env()
print(f"scene {a.config}: {sd.counts} prep {time.time()-t0:.2f}s", flush=True)
r = Renderer(0)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*env)
r.resize(W, H)
print("device", r.device_info(), flush=True)
fp = cf.frame_params(W, H, max_bounce=a.max_bounce, flags=a.flags)
ro = cf.rand_origins(a.frames + 1 + max(64, a.count_frames))
rays_total = r.render(fp, ro[:1])["rays"]
r.reset_stats()
t = time.time()
k = 1
while k < a.frames + 1:
    n = min(a.per_launch, a.frames + 1 - k)
    r.render_async(fp, ro[k:k + n])
    k += n
st = r.stats()
wall = time.time() - t
rays_total += st["rays"]
ms = st["kernel_ms"] / a.frames
print(f"{a.config} {W}x{H} mb={a.max_bounce} flags={a.flags}: {ms:.2f} ms/frame (kernel), wall {wall*1000/a.frames:.2f} ms/frame, "
      f"{st['rays']/st['kernel_ms']/1e3:.1f} Mrays/s, rays/frame {st['rays']/a.frames/1e6:.2f} M", flush=True)
fpc = cf.frame_params(W, H, max_bounce=a.max_bounce, flags=RT_FLAG_COUNT_VISITS | a.flags)
r.reset_stats()
r.render(fpc, ro[-a.count_frames:])
st = r.stats()
rays_total += st["rays"]
print("visits per ray: internal %.1f leaf %.1f tri %.1f; trace loop iters/wave-pass avg %.0f max %d (%d launches)" % (
      st["internal_pops"] / st["rays"], st["leaf_pops"] / st["rays"], st["tri_tests"] / st["rays"],
      st["trace_iters"] / max(1, st["trace_launches"]) / 3072, st["trace_iters_max"], st["trace_launches"]), flush=True)
print(f"rays_total {rays_total}", flush=True)  # every render of the run (tools/pmc_cmp.py: per ray)
