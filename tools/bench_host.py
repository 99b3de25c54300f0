#!/usr/bin/env python3
"""Host scene preparation timings: OBJ load + normals (H1), placement
(H2), SAH BVH (H3, literal restatement vs the faithful parallel build), encodings (H4), HDR
decode + cache (H5/H6).  OBJ text comes from /root/reference when present (this container),
otherwise the pre-parsed assets/*.npz (H1 then times only the mesh build).

    python tools/bench_host.py [--config C3]
"""
import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

STAGES = r'''
import json, os, sys, time
from pathlib import Path
sys.path.insert(0, sys.argv[1])
from rtamd import configs as cf, scene_lib as sl
name, ref = sys.argv[2], Path("/root/reference/resources/objects")
out = {}
t = time.perf_counter()
meshes = []
for o in cf.CONFIGS[name].objects:
    obj = ref / (o.mesh + ".obj")
    meshes.append(sl.Mesh.load(str(obj)) if obj.exists() else cf.load_mesh(o.mesh))
out["H1_obj_load_s"] = time.perf_counter() - t
out["H1_source"] = "obj text" if (ref / (cf.CONFIGS[name].objects[-1].mesh + ".obj")).exists() else "npz"
t = time.perf_counter()
s = sl.Scene()
for o, m in zip(cf.CONFIGS[name].objects, meshes):
    s.add_mesh(m, cf.MATERIALS[o.material], o.rotate, o.translate, o.scale, o.smooth)
out["H2_place_s"] = time.perf_counter() - t
t = time.perf_counter(); s.build_bvh(8); out["H3_bvh_s"] = time.perf_counter() - t
t = time.perf_counter(); s.encode(); s.export_soa(); out["H4_encode_s"] = time.perf_counter() - t
t = time.perf_counter(); img = sl.load_hdr(str(cf.ASSET_DIR / cf.HDR_ASSET)); out["H5_hdr_s"] = time.perf_counter() - t
t = time.perf_counter(); sl.hdr_cache(img); out["H6_cache_s"] = time.perf_counter() - t
out["counts"] = s.counts()
print(json.dumps(out))
'''


def run(name: str, literal: bool) -> dict:
    env = dict(os.environ, RTS_BVH_LITERAL="1" if literal else "0")
    p = subprocess.run([sys.executable, "-c", STAGES, str(ROOT / "opengl-ray-tracing-framework_amd"), name],
                       env=env, capture_output=True, text=True, check=True)
    return json.loads(p.stdout)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    a = ap.parse_args()
    lit, fast = run(a.config, True), run(a.config, False)
    res = {"config": a.config, "threads": os.cpu_count(), "literal": lit, "fast": fast,
           "bvh_speedup": round(lit["H3_bvh_s"] / fast["H3_bvh_s"], 2)}
    print(json.dumps(res, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
