#!/usr/bin/env python3
"""Drive the interactive loop headless (rtamd.interactive: Camera.h + main.cpp's render loop):
a scripted walk (hold W, strafe, right-button drags, GUI edits) at one frame per loop pass, the
reference's interactive mode.  Reports the per-frame latency of each phase of the script and
writes the displayed image at the end of each phase.

    python tools/interactive_demo.py --config C3 --frames 30 --out gpurun_out/interactive
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

from rtamd import configs as cf  # noqa: E402
from rtamd import interactive as ia  # noqa: E402
from rtamd import scene_lib as sl  # noqa: E402
from rtamd.renderer import Renderer  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="C3")
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--frames", type=int, default=30, help="loop passes per script phase")
ap.add_argument("--out", default="")
ap.add_argument("--png", action="store_true", help="write the displayed image of each phase under --out")
ap.add_argument("--no-display", action="store_true", help="skip the per-frame 8-bit read-back")
ap.add_argument("--in-flight", type=int, default=1,
                help="frames in flight (Session frames_in_flight: the GL frame queue; images unchanged)")
a = ap.parse_args()

cfg = cf.CONFIGS[a.config]
W, H = a.width or cfg.width, a.height or cfg.height
sd = cf.config_scene(a.config)
r = Renderer(0)
r.set_scene_soa(sd.soa, sd.nodes)
r.set_env(*cf.load_env())
s = ia.Session(r, W, H, frames_in_flight=a.in_flight)
dt = 1.0 / 60.0
phases = [
    ("still", lambda k: ia.Input()),
    ("walk_forward", lambda k: ia.Input(keys=["w"])),
    ("strafe_up", lambda k: ia.Input(keys=["d", "q"])),
    ("drag", lambda k: ia.Input(mouse=[(500 + 4 * k, 300 - k, True)])),
    ("gui_env_off", lambda k: ia.Input(gui={"enable_env_map": False}) if k == 0 else ia.Input()),
    ("still_after", lambda k: ia.Input()),
]
for _ in range(max(1, a.in_flight)):  # first passes: allocations (every pipeline set), code objects
    s.tick(delta_time=dt, display=not a.no_display)
s.flush()
report = {"config": a.config, "width": W, "height": H, "frames_per_phase": a.frames, "frames_in_flight": a.in_flight,
          "phases": {}}
for name, make in phases:
    r.synchronize()
    t0 = time.perf_counter()
    out = None
    for k in range(a.frames):
        out = s.tick(make(k), delta_time=dt, display=not a.no_display) or out
    out = (s.flush() or [out])[-1]  # the phase's last displayed frame (the queue drained)
    r.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / a.frames
    report["phases"][name] = {"ms_per_frame": round(ms, 3), "fps": round(1e3 / ms, 1), "loop_num": out["loop_num"]}
    print(f"{name:14s} {ms:7.3f} ms/frame ({1e3 / ms:6.1f} fps), LoopNum {out['loop_num']}", flush=True)
    if a.out and a.png and "image" in out:
        Path(a.out).mkdir(parents=True, exist_ok=True)
        sl.write_png(str(Path(a.out) / f"{a.config}_{name}.png"), out["image"])
if a.out:
    Path(a.out).mkdir(parents=True, exist_ok=True)
    (Path(a.out) / f"{a.config}_interactive.json").write_text(json.dumps(report, indent=1))
