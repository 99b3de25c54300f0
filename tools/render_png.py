#!/usr/bin/env python3
"""Render a config progressively and save the displayed image (the reference's render loop,
main.cpp:165-253, + SaveFrame, Utility.h:19-30), headless.

    python tools/render_png.py --config C3 --spp 64 --out gpurun_out/C3_64spp.png
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

from rtamd import configs as cf  # noqa: E402
from rtamd import scene_lib as sl  # noqa: E402
from rtamd.renderer import RT_DISPLAY_GAMMA, RT_DISPLAY_TONEMAP, Renderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--spp", type=int, default=64)
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--no-tonemap", action="store_true", help="enableToneMapping off: the screen blit")
ap.add_argument("--no-gamma", action="store_true", help="enableGammaCorrection off")
ap.add_argument("--brdf", action="store_true", help="enableBSDF off")
ap.add_argument("--out", default="render.png")
a = ap.parse_args()

cfg = cf.CONFIGS[a.config]
W, H = a.width or cfg.width, a.height or cfg.height
sd = cf.config_scene(a.config)
r = Renderer(0)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*cf.load_env())
r.resize(W, H)
fp = cf.frame_params(W, H, enable_bsdf=not a.brdf)
t = time.time()
st = r.render(fp, cf.rand_origins(a.spp))
dt = time.time() - t
flags = (0 if a.no_tonemap else RT_DISPLAY_TONEMAP) | (0 if a.no_gamma else RT_DISPLAY_GAMMA)
img = r.tonemap(flags)
Path(a.out).parent.mkdir(parents=True, exist_ok=True)
sl.write_png(a.out, img)
print(f"{a.config} {W}x{H} {a.spp} spp in {dt:.2f} s ({st['rays'] / dt / 1e6:.0f} Mrays/s) -> {a.out}")
