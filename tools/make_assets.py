#!/usr/bin/env python3
"""Write the compact scene assets under assets/ from the reference's resources.

The GPU box receives only this repository, so the meshes travel as the raw OBJ parse
result (positions, file normals, polygon faces; correctly-rounded float parse) in .npz,
and the HDR environment as the original Radiance file.  Run in the build container:

    python tools/make_assets.py [--reference /root/reference]
"""
import argparse
import shutil
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

from rtamd import scene_lib as sl  # noqa: E402

MESHES = ("floor", "bunny_4000", "loong_100000", "sphere")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    ref = Path(args.reference)
    out = ROOT / "assets"
    out.mkdir(exist_ok=True)
    for name in MESHES:
        raw = sl.parse_obj_raw(str(ref / "resources" / "objects" / f"{name}.obj"), 0)
        np.savez_compressed(out / f"{name}.npz", positions=raw.positions, normals=raw.normals,
                            face_sizes=raw.face_sizes, pos_index=raw.pos_index, nrm_index=raw.nrm_index)
        print(f"{name}: {len(raw.positions)} positions, {len(raw.face_sizes)} faces")
    hdr = ref / "resources" / "textures" / "hdr" / "peppermint_powerplant_1k.hdr"
    shutil.copyfile(hdr, out / hdr.name)
    print(f"copied {hdr.name}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
