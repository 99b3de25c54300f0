#!/usr/bin/env python3
"""Generate the committed fixtures under tests/golden/ (run in the build container).

* rand_origins.json   randOrigin_k for k = 1..16384 (glibc srand(20221002), main.cpp:190)
* hdr_ref.json        the reference HDRLoader's decode of peppermint_powerplant_1k.hdr, from
                      oracle/_ref/ref_hdr_dump (thirdparty/hdrloader/hdrloader.cpp compiled from
                      its own sources by oracle/Makefile): size, checksums, sampled texels
* bvh_counts.json     node / leaf / depth counts measured from the reference BVH.h (SURVEY.md
                      §8(c) table) — copied, not recomputed
* scene_hashes.json   sha256 of our encoded C2/C3 arrays (regression of the host pipeline)
* oracle_*.npy        small oracle renders (regression of the oracle itself)
"""
import hashlib
import json
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
GOLD = ROOT / "tests" / "golden"

from rtamd import configs as cf  # noqa: E402
from rtamd import scene_lib as sl  # noqa: E402

HDR_SAMPLE_IDX = np.random.default_rng(7).integers(0, 1024 * 512, 256)
ORACLE_GOLDEN = [("C2", 48, 27, 2), ("C3", 48, 27, 2), ("C4", 48, 27, 2)]


def read_ref_dump(path: Path):
    raw = path.read_bytes()
    w, h = np.frombuffer(raw[:8], np.int32)
    img = np.frombuffer(raw[8:], np.float32).reshape(h, w, 3)
    return img


def main() -> int:
    GOLD.mkdir(parents=True, exist_ok=True)
    ro = sl.cpu_rand_origins(cf.RAND_SEED, 16384)
    (GOLD / "rand_origins.json").write_text(json.dumps({
        "note": "randOrigin_k = 674764*(rand()/(RAND_MAX+1.0)+1) after glibc srand(20221002), k=1..16384 "
                "(main.cpp:190, src/core/Utility.h:11-17); float32 bit patterns",
        "seed": cf.RAND_SEED, "bits": [int(x) for x in ro.view(np.uint32)]}))

    ref_bin = ROOT / "oracle" / "_ref" / "ref_hdr_dump"
    hdr_path = ROOT / "assets" / cf.HDR_ASSET
    if ref_bin.exists():
        with tempfile.TemporaryDirectory() as td:
            out = Path(td) / "hdr.bin"
            subprocess.run([str(ref_bin), str(hdr_path), str(out)], check=True)
            img = read_ref_dump(out)
        flat = img.reshape(-1, 3)
        (GOLD / "hdr_ref.json").write_text(json.dumps({
            "source": "oracle/_ref/ref_hdr_dump = reference thirdparty/hdrloader/hdrloader.cpp (clang, -O2)",
            "width": int(img.shape[1]), "height": int(img.shape[0]),
            "sum_f64": float(img.astype(np.float64).sum()), "max": float(img.max()),
            "pixel0": [float(v) for v in flat[0]],
            "sha256": hashlib.sha256(img.tobytes()).hexdigest(),
            "sample_index": [int(i) for i in HDR_SAMPLE_IDX],
            "sample_bits": [[int(b) for b in flat[i].view(np.uint32)] for i in HDR_SAMPLE_IDX]}, indent=0))
        print("hdr_ref.json written")
    else:
        print("oracle/_ref not built: hdr_ref.json left as is")

    (GOLD / "bvh_counts.json").write_text(json.dumps({
        "source": "SURVEY.md §8(c): src/core/BVH.h compiled verbatim in the survey container (leaf size 8)",
        "raw_bunny_4000": {"triangles": 4968, "nodes": 1740, "leaves": 870},
        "raw_loong_100000": {"triangles": 100000, "nodes": 35420, "leaves": 17710},
        "C2_scene": {"triangles": 4970, "nodes": 1740, "max_depth": 14},
        "C3_scene": {"triangles": 100002, "nodes": 35346, "max_depth": 22}}, indent=1))

    hashes = {}
    for name in ("C2", "C3"):
        sd = cf.config_scene(name)
        hashes[name] = {"tri_enc": hashlib.sha256(sd.tri_enc.tobytes()).hexdigest(),
                        "node_enc": hashlib.sha256(sd.node_enc.tobytes()).hexdigest()}
    (GOLD / "scene_hashes.json").write_text(json.dumps(hashes, indent=1))

    import oracle as orc
    env = cf.load_env()
    for name, W, H, n in ORACLE_GOLDEN:
        sd = cf.config_scene(name)
        fp = cf.frame_params(W, H)
        r = cf.rand_origins(n)
        frames = [cf.oracle_frame_params(fp, k + 1, r[k]) for k in range(n)]
        img, cnt = orc.render(orc.OracleScene(sd.tri_enc, sd.node_enc, env[0], env[1]), frames, W, H)
        np.save(GOLD / f"oracle_{name}_{W}x{H}_f{n}.npy", img)
        (GOLD / f"oracle_{name}_{W}x{H}_f{n}.json").write_text(json.dumps(cnt))
        print(name, cnt)
    return 0


if __name__ == "__main__":
    sys.exit(main())
