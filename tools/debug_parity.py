#!/usr/bin/env python3
"""Development aid: locate GPU-vs-oracle divergences (by bounce depth, culling, pixel)."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
sys.path.insert(0, str(ROOT / "tests"))
from helpers import bit_mismatch, frames_for, gpu_render, oracle_render  # noqa: E402
from rtamd import configs as cf  # noqa: E402
from rtamd.renderer import RT_FLAG_NO_CULL, Renderer  # noqa: E402

env = cf.load_env()
r = Renderer(0)
W, H = 96, 54
for name in sys.argv[1:] or ["C2"]:
    sd = cf.config_scene(name)
    for mb in (0, 1, 2, 8):
        for flags in (0, RT_FLAG_NO_CULL):
            fp = cf.frame_params(W, H, max_bounce=mb, flags=flags)
            ro, frames = frames_for(fp, 1, 1)
            ref, cnt = oracle_render(sd, env, W, H, frames)
            img, st = gpu_render(r, sd, env, W, H, fp, ro)
            frac, diff = bit_mismatch(img, ref)
            ys, xs = np.nonzero(diff)
            print(f"{name} mb={mb} flags={flags}: mismatch {frac:.4%} rays gpu {st['rays']} orc {cnt['rays']}", flush=True)
            for y, x in list(zip(ys, xs))[:4]:
                print(f"   px ({x},{y}) gpu {img[y, x]} orc {ref[y, x]}")
