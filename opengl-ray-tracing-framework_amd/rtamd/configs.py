"""The reference's scenes and BASELINE.json configs C1-C5 as concrete inputs.

Materials: src/core/Scene.h:53-109.  Object placements: src/core/Scene.h:116-143.
Camera defaults: src/core/RenderSettings.h:18-20 (position (0,0,7), rotation (-87.78,-14,0)),
zoom 30 (src/core/Camera.h:23,:59).  Render settings: src/core/RenderSettings.h:81-90.
randOrigin_k: main.cpp:190 with glibc rand() after srand(20221002).

Meshes load from the compact assets under ``assets/`` (raw OBJ parse results written by
tools/make_assets.py from /root/reference/resources/objects), so the GPU box needs no
reference checkout.  ``panther_100000.obj`` is absent from the reference
(.MISSING_LARGE_BLOBS:1): C4/C5 use loong geometry with the panther transform/material,
labelled "panther-proxy".
"""
from __future__ import annotations

import dataclasses
import json
from functools import lru_cache
from typing import List, Optional

import numpy as np

from . import scene_lib as sl
from ._paths import ASSET_DIR, GOLDEN_DIR
from .renderer import FrameParams

f32 = np.float32


def _c(*v):
    return tuple(float(f32(x)) for x in v)


MATERIALS = {
    "plane": sl.Material(base_color=_c(0.73, 0.73, 0.73), specular=1.0, ior=1.79, metallic=0.2),
    "white": sl.Material(base_color=_c(0.73, 0.73, 0.73), roughness=0.5, specular=0.5),
    "jade": sl.Material(base_color=_c(0.55, 0.78, 0.55), specular=1.0, ior=1.79, subsurface=1.0),
    "golden": sl.Material(base_color=_c(0.75, 0.7, 0.15), roughness=0.05, specular=1.0, metallic=1.0),
    "copper": sl.Material(base_color=(float(f32(238.0) / f32(255.0)), float(f32(158.0) / f32(255.0)),
                                      float(f32(137.0) / f32(255.0))),
                          roughness=0.2, specular=1.0, ior=1.21901, metallic=1.0),
    "glass": sl.Material(base_color=(1, 1, 1), specular=1.0, transmission=1.0, ior=1.5, roughness=0.02),
    "brown_glass": sl.Material(base_color=(1, 1, 1), medium_type=1, medium_color=_c(0.905, 0.63, 0.3),
                               medium_density=1, specular=1.0, transmission=0.957, ior=1.45, roughness=0.1),
    "tear_glass": sl.Material(base_color=(1, 1, 1), medium_color=_c(0.085, 0.917, 0.848), medium_density=1,
                              medium_type=1, specular=1.0, transmission=0.917, ior=1.45),
    "tear_glass_emissive": sl.Material(base_color=(1, 1, 1), medium_color=_c(0.085, 0.917, 0.848),
                                       medium_density=0.25, medium_type=3, specular=1.0, transmission=0.917,
                                       ior=1.45),
}


@dataclasses.dataclass(frozen=True)
class Obj:
    mesh: str          # asset name
    material: object   # a MATERIALS key or an sl.Material
    rotate: tuple
    translate: tuple
    scale: tuple
    smooth: bool


FLOOR = Obj("floor", "plane", (0, 0, 0), (2.2, -2, 3), (14, 7, 7), False)          # Scene.h:116-120
BUNNY = Obj("bunny_4000", "jade", (0, 0, 0), (2.2, -2.5, 3), (2, 2, 2), False)      # Scene.h:122-126
LOONG = Obj("loong_100000", "copper", (0, 0, 0), (2, -2, 3), (3.5, 3.5, 3.5), True) # Scene.h:134-138
PANTHER_PROXY = Obj("loong_100000", "brown_glass", (0, -30, 0), (0.8, -2.2, 5), (4.5, 4.5, 4.5), True)  # :140-143


@dataclasses.dataclass(frozen=True)
class Config:
    name: str
    objects: tuple
    width: int
    height: int
    spp: int
    gpus: int
    note: str = ""


CONFIGS = {
    "C1": Config("C1", (FLOOR, BUNNY), 1280, 720, 0, 0, "host prep only (bunny_4000)"),
    "C2": Config("C2", (FLOOR, BUNNY), 1280, 720, 256, 1, "bunny_4000 jade subsurface"),
    "C3": Config("C3", (FLOOR, LOONG), 1920, 1080, 1024, 1, "loong_100000 copper metallic (north star)"),
    "C4": Config("C4", (FLOOR, PANTHER_PROXY), 1920, 1080, 1024, 8, "panther-proxy absorbing glass"),
    "C5": Config("C5", (FLOOR, BUNNY, LOONG, PANTHER_PROXY), 3840, 2160, 4096, 8,
                 "merged bunny+loong+panther-proxy, HDR env IS"),
}

CAMERA_POSITION = (0.0, 0.0, 7.0)
CAMERA_ROTATION = (-87.78, -14.0, 0.0)
CAMERA_ZOOM = 30.0
RAND_SEED = 20221002
HDR_ASSET = "peppermint_powerplant_1k.hdr"


@lru_cache(maxsize=None)
def load_raw_mesh(name: str) -> sl.RawObj:
    with np.load(ASSET_DIR / f"{name}.npz", allow_pickle=False) as z:
        return sl.RawObj(z["positions"], z["normals"], z["face_sizes"], z["pos_index"], z["nrm_index"])


@lru_cache(maxsize=None)
def load_mesh(name: str) -> sl.Mesh:
    return sl.Mesh.from_raw(load_raw_mesh(name))


@lru_cache(maxsize=None)
def load_env():
    img = sl.load_hdr(str(ASSET_DIR / HDR_ASSET))
    return img, sl.hdr_cache(img)


@dataclasses.dataclass
class SceneData:
    name: str
    counts: dict
    tri_enc: np.ndarray   # (n, 14, 3) Triangle_encoded
    node_enc: np.ndarray  # (nn, 4, 3) BVHNode_encoded
    soa: dict
    nodes: dict
    ranges: List[tuple]   # pre-BVH triangle range per object


def build_scene(objects, leaf_size: int = 8) -> SceneData:
    """InitMesh + EncodedBVHandTriangles (src/core/Scene.h:111-257) for a list of Obj."""
    s = sl.Scene()
    ranges = []
    for o in objects:
        mat = o.material if isinstance(o.material, sl.Material) else MATERIALS[o.material]
        ranges.append(s.add_mesh(load_mesh(o.mesh), mat, o.rotate, o.translate, o.scale, o.smooth))
    s.build_bvh(leaf_size)
    tri, nodes = s.encode()
    return SceneData("custom", s.counts(), tri, nodes, s.export_soa(), s.nodes(), ranges)


@lru_cache(maxsize=None)
def config_scene(name: str) -> SceneData:
    sd = build_scene(CONFIGS[name].objects)
    sd.name = name
    return sd


def frame_params(width: int, height: int, **overrides) -> FrameParams:
    cam = sl.camera(CAMERA_ROTATION[0], CAMERA_ROTATION[1], CAMERA_ZOOM, float(f32(width) / f32(height)))
    fp = FrameParams(position=CAMERA_POSITION, front=cam["front"], right=cam["right"], up=cam["up"],
                     left_bottom_corner=cam["left_bottom_corner"], half_h=cam["half_h"], half_w=cam["half_w"])
    for k, v in overrides.items():
        setattr(fp, k, v)
    return fp


@lru_cache(maxsize=1)
def _fixture_bits() -> np.ndarray:
    with open(GOLDEN_DIR / "rand_origins.json") as f:
        return np.array(json.load(f)["bits"], dtype=np.uint32)


def rand_origins(n: int, offset: int = 0) -> np.ndarray:
    """randOrigin for frames offset+1 .. offset+n after glibc srand(20221002) (main.cpp:190), any
    length: generated by librtscene's in-tree restatement of glibc rand() (rts_glibc_rand), and
    the part that overlaps the committed 16,384-frame fixture (made with the libc's own rand())
    must equal it bit for bit."""
    if n < 0 or offset < 0:
        raise ValueError("rand_origins: n and offset must be >= 0")
    out = sl.cpu_rand_origins(RAND_SEED, offset + n)[offset:]
    bits = _fixture_bits()
    k = max(0, min(len(bits), offset + n) - offset)
    if k and not np.array_equal(out[:k].view(np.uint32), bits[offset:offset + k]):
        raise RuntimeError("randOrigin generator disagrees with tests/golden/rand_origins.json")
    return out


def oracle_frame_params(fp: FrameParams, loop_num: int, rand_origin: float) -> dict:
    d = dataclasses.asdict(fp)
    d["loop_num"] = loop_num
    d["rand_origin"] = float(rand_origin)
    return d
