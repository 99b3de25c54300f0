"""ctypes bindings of librtscene.so (include/rt_scene.h): the reference's host pipeline.

Python mirror of the reference's scene-assembly calls (src/core/Scene.h:35-257):
``Mesh.load`` ~ ``Model(path)``, ``Scene.add_mesh`` ~ ``getTriangle(...)``,
``Scene.build_bvh`` ~ ``buildBVHwithSAH(...)``, ``Scene.encode`` ~
``EncodedBVHandTriangles()``, ``load_hdr``/``hdr_cache`` ~ ``InitHdrEnvMap()``.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
from typing import Optional, Sequence

import numpy as np

from ._paths import lib_path

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)


class RtsMaterial(C.Structure):
    _fields_ = [
        ("emissive", C.c_float * 3),
        ("base_color", C.c_float * 3),
        ("subsurface", C.c_float), ("metallic", C.c_float), ("specular", C.c_float),
        ("specular_tint", C.c_float), ("roughness", C.c_float), ("anisotropic", C.c_float),
        ("sheen", C.c_float), ("sheen_tint", C.c_float), ("clearcoat", C.c_float),
        ("clearcoat_gloss", C.c_float), ("ior", C.c_float), ("transmission", C.c_float),
        ("medium_color", C.c_float * 3),
        ("medium_type", C.c_float), ("medium_density", C.c_float), ("medium_anisotropy", C.c_float),
    ]


@dataclasses.dataclass
class Material:
    """src/core/Material.h:25-46 with the reference defaults."""
    emissive: Sequence[float] = (0.0, 0.0, 0.0)
    base_color: Sequence[float] = (1.0, 1.0, 1.0)
    subsurface: float = 0.0
    metallic: float = 0.0
    specular: float = 0.0
    specular_tint: float = 0.0
    roughness: float = 0.0
    anisotropic: float = 0.0
    sheen: float = 0.0
    sheen_tint: float = 0.0
    clearcoat: float = 0.0
    clearcoat_gloss: float = 0.0
    ior: float = 1.0
    transmission: float = 0.0
    medium_color: Sequence[float] = (1.0, 1.0, 1.0)
    medium_type: float = 0.0
    medium_density: float = 0.0
    medium_anisotropy: float = 0.0

    def to_c(self) -> RtsMaterial:
        m = RtsMaterial()
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            if isinstance(v, (tuple, list)):
                arr = getattr(m, f.name)
                for i in range(3):
                    arr[i] = float(np.float32(v[i]))
            else:
                setattr(m, f.name, float(np.float32(v)))
        return m

    def texels(self) -> np.ndarray:
        """The 24 material floats of Triangle_encoded texels 6..13 (src/core/Triangle.h:31-38)."""
        return np.array(list(self.emissive) + list(self.base_color) + [
            self.subsurface, self.metallic, self.specular, self.specular_tint, self.roughness,
            self.anisotropic, self.sheen, self.sheen_tint, self.clearcoat, self.clearcoat_gloss,
            self.ior, self.transmission] + list(self.medium_color) + [
            self.medium_type, self.medium_density, self.medium_anisotropy], dtype=np.float32)


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        L = C.CDLL(str(lib_path("librtscene.so")))
        vp = C.c_void_p
        L.rts_obj_load.argtypes = [C.c_char_p, C.c_int, C.POINTER(vp)]
        L.rts_obj_parse_raw.argtypes = [C.c_char_p, C.c_int, _i32p, _i32p, _i32p, _i32p, _f32p, _f32p, _i32p,
                                        _i32p, _i32p]
        L.rts_mesh_from_raw.argtypes = [_f32p, C.c_int, _f32p, C.c_int, _i32p, C.c_int, _i32p, _i32p,
                                        C.POINTER(vp)]
        L.rts_mesh_counts.argtypes = [vp, _i32p, _i32p]
        L.rts_mesh_data.argtypes = [vp, _f32p, _f32p, _i32p]
        L.rts_mesh_free.argtypes = [vp]
        L.rts_mesh_free.restype = None
        L.rts_scene_create.argtypes = [C.POINTER(vp)]
        L.rts_scene_free.argtypes = [vp]
        L.rts_scene_free.restype = None
        L.rts_scene_add_mesh.argtypes = [vp, vp, C.POINTER(RtsMaterial), _f32p, _f32p, _f32p, C.c_int, _i32p]
        L.rts_scene_add_triangles.argtypes = [vp, _f32p, C.c_int, C.POINTER(RtsMaterial), _i32p]
        L.rts_scene_build_bvh.argtypes = [vp, C.c_int]
        L.rts_scene_counts.argtypes = [vp, _i32p, _i32p, _i32p, _i32p]
        L.rts_scene_encode.argtypes = [vp, _f32p, _f32p]
        L.rts_scene_nodes.argtypes = [vp, _i32p, _i32p, _i32p, _i32p, _f32p, _f32p]
        L.rts_scene_export_soa.argtypes = [vp, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _i32p,
                                           C.POINTER(RtsMaterial), _i32p]
        L.rts_scene_set_material.argtypes = [vp, C.c_int, C.c_int, C.POINTER(RtsMaterial)]
        L.rts_scene_post_bvh_index.argtypes = [vp, _i32p]
        L.rts_hdr_load.argtypes = [C.c_char_p, _i32p, _i32p, C.POINTER(_f32p)]
        L.rts_hdr_cache.argtypes = [_f32p, C.c_int, C.c_int, _f32p]
        L.rts_free.argtypes = [vp]
        L.rts_free.restype = None
        L.rts_camera.argtypes = [C.c_float, C.c_float, C.c_float, C.c_float, _f32p]
        L.rts_cpu_rand_origins.argtypes = [C.c_uint, C.c_int, _f32p]
        L.rts_glibc_rand.argtypes = [C.c_uint, C.c_int, C.POINTER(C.c_int)]
        L.rts_write_png.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_uint8)]
        L.rts_tri_filter.argtypes = [_f32p, C.c_int, _f32p, C.POINTER(C.c_double), _i32p]
        _lib = L
    return _lib


def _fp(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(_f32p)


def _ip(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(_i32p)


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with rts error {rc}")


@dataclasses.dataclass
class RawObj:
    """OBJ data as parsed: positions, file normals, polygon faces (0-based indices)."""
    positions: np.ndarray
    normals: np.ndarray
    face_sizes: np.ndarray
    pos_index: np.ndarray
    nrm_index: np.ndarray


def parse_obj_raw(path: str, parse_mode: int = 0) -> RawObj:
    L = lib()
    n = [C.c_int32() for _ in range(4)]
    _check(L.rts_obj_parse_raw(str(path).encode(), parse_mode, *[C.byref(x) for x in n],
                               None, None, None, None, None), "rts_obj_parse_raw(sizes)")
    npos, nnrm, nf, ni = (x.value for x in n)
    raw = RawObj(np.zeros((npos, 3), np.float32), np.zeros((nnrm, 3), np.float32),
                 np.zeros(nf, np.int32), np.zeros(ni, np.int32), np.zeros(ni, np.int32))
    _check(L.rts_obj_parse_raw(str(path).encode(), parse_mode, *[C.byref(x) for x in n],
                               _fp(raw.positions), _fp(raw.normals), _ip(raw.face_sizes), _ip(raw.pos_index),
                               _ip(raw.nrm_index)), "rts_obj_parse_raw")
    return raw


class Mesh:
    """A post-processed model (assimp Triangulate | GenSmoothNormals semantics)."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle)

    @classmethod
    def load(cls, path: str, parse_mode: int = 0) -> "Mesh":
        h = C.c_void_p()
        _check(lib().rts_obj_load(str(path).encode(), parse_mode, C.byref(h)), f"rts_obj_load({path})")
        return cls(h.value)

    @classmethod
    def from_raw(cls, raw: RawObj) -> "Mesh":
        h = C.c_void_p()
        pos = np.ascontiguousarray(raw.positions, np.float32)
        nrm = np.ascontiguousarray(raw.normals, np.float32)
        fs = np.ascontiguousarray(raw.face_sizes, np.int32)
        pi = np.ascontiguousarray(raw.pos_index, np.int32)
        ni = np.ascontiguousarray(raw.nrm_index, np.int32)
        _check(lib().rts_mesh_from_raw(_fp(pos), len(pos), _fp(nrm) if len(nrm) else None, len(nrm), _ip(fs), len(fs),
                                       _ip(pi), _ip(ni), C.byref(h)), "rts_mesh_from_raw")
        return cls(h.value)

    def data(self):
        nv, ni = C.c_int32(), C.c_int32()
        _check(lib().rts_mesh_counts(self._h, C.byref(nv), C.byref(ni)), "rts_mesh_counts")
        pos = np.zeros((nv.value, 3), np.float32)
        nrm = np.zeros((nv.value, 3), np.float32)
        idx = np.zeros(ni.value, np.int32)
        _check(lib().rts_mesh_data(self._h, _fp(pos), _fp(nrm), _ip(idx)), "rts_mesh_data")
        return pos, nrm, idx

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None and self._h.value:
            _lib.rts_mesh_free(self._h)
            self._h = C.c_void_p()


class Scene:
    """Triangle list + SAH BVH (src/core/RenderSettings.h:502 ``triangles`` + BVH.h)."""

    def __init__(self):
        h = C.c_void_p()
        _check(lib().rts_scene_create(C.byref(h)), "rts_scene_create")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None and self._h.value:
            _lib.rts_scene_free(self._h)
            self._h = C.c_void_p()

    def add_mesh(self, mesh: Mesh, material: Material, rotate=(0, 0, 0), translate=(0, 0, 0), scale=(1, 1, 1),
                 smooth: bool = False):
        r = np.asarray(rotate, np.float32)
        t = np.asarray(translate, np.float32)
        s = np.asarray(np.broadcast_to(np.asarray(scale, np.float32), (3,)), np.float32).copy()
        rng = np.zeros(2, np.int32)
        m = material.to_c()
        _check(lib().rts_scene_add_mesh(self._h, mesh._h, C.byref(m), _fp(r), _fp(t), _fp(s), int(smooth), _ip(rng)),
               "rts_scene_add_mesh")
        return int(rng[0]), int(rng[1])

    def add_triangles(self, positions: np.ndarray, material: Material):
        p = np.ascontiguousarray(positions, np.float32).reshape(-1, 9)
        rng = np.zeros(2, np.int32)
        m = material.to_c()
        _check(lib().rts_scene_add_triangles(self._h, _fp(p), len(p), C.byref(m), _ip(rng)), "rts_scene_add_triangles")
        return int(rng[0]), int(rng[1])

    def build_bvh(self, leaf_size: int = 8) -> None:
        _check(lib().rts_scene_build_bvh(self._h, leaf_size), "rts_scene_build_bvh")

    def counts(self):
        v = [C.c_int32() for _ in range(4)]
        _check(lib().rts_scene_counts(self._h, *[C.byref(x) for x in v]), "rts_scene_counts")
        return dict(zip(("n_triangles", "n_nodes", "max_depth", "n_leaves"), (x.value for x in v)))

    def encode(self):
        c = self.counts()
        tri = np.zeros((c["n_triangles"], 14, 3), np.float32)
        nodes = np.zeros((c["n_nodes"], 4, 3), np.float32)
        _check(lib().rts_scene_encode(self._h, _fp(tri), _fp(nodes) if c["n_nodes"] else None), "rts_scene_encode")
        return tri, nodes

    def nodes(self):
        nn = self.counts()["n_nodes"]
        out = {k: np.zeros(nn, np.int32) for k in ("left", "right", "n", "index")}
        aa = np.zeros((nn, 3), np.float32)
        bb = np.zeros((nn, 3), np.float32)
        _check(lib().rts_scene_nodes(self._h, _ip(out["left"]), _ip(out["right"]), _ip(out["n"]), _ip(out["index"]),
                                     _fp(aa), _fp(bb)), "rts_scene_nodes")
        out["aa"], out["bb"] = aa, bb
        return out

    def export_soa(self):
        nt = self.counts()["n_triangles"]
        arr = {k: np.zeros((nt, 3), np.float32) for k in ("p1", "p2", "p3", "n1", "n2", "n3")}
        mid = np.zeros(nt, np.int32)
        nm = C.c_int32()
        _check(lib().rts_scene_export_soa(self._h, *(None for _ in range(7)), None, C.byref(nm)), "export_soa(count)")
        mats = (RtsMaterial * max(nm.value, 1))()
        _check(lib().rts_scene_export_soa(self._h, *(_fp(arr[k]) for k in ("p1", "p2", "p3", "n1", "n2", "n3")),
                                          _ip(mid), mats, C.byref(nm)), "rts_scene_export_soa")
        arr["material_id"] = mid
        arr["materials"] = np.ctypeslib.as_array(
            C.cast(mats, C.POINTER(C.c_float)), shape=(max(nm.value, 1), 24))[: nm.value].copy()
        return arr

    def set_material(self, first: int, count: int, material: Material) -> None:
        m = material.to_c()
        _check(lib().rts_scene_set_material(self._h, first, count, C.byref(m)), "rts_scene_set_material")

    def post_bvh_index(self) -> np.ndarray:
        out = np.zeros(self.counts()["n_triangles"], np.int32)
        _check(lib().rts_scene_post_bvh_index(self._h, _ip(out)), "rts_scene_post_bvh_index")
        return out


def load_hdr(path: str) -> np.ndarray:
    """Radiance .hdr -> float32 (H, W, 3), row 0 = file's first scanline (HDRLoader order)."""
    L = lib()
    w, h = C.c_int32(), C.c_int32()
    p = _f32p()
    _check(L.rts_hdr_load(str(path).encode(), C.byref(w), C.byref(h), C.byref(p)), f"rts_hdr_load({path})")
    try:
        img = np.ctypeslib.as_array(p, shape=(h.value, w.value, 3)).copy()
    finally:
        L.rts_free(C.cast(p, C.c_void_p))
    return img


def hdr_cache(img: np.ndarray) -> np.ndarray:
    img = np.ascontiguousarray(img, np.float32)
    h, w, _ = img.shape
    out = np.zeros_like(img)
    _check(lib().rts_hdr_cache(_fp(img), w, h, _fp(out)), "rts_hdr_cache")
    return out


def camera(yaw: float, pitch: float, zoom: float, ratio: float) -> dict:
    out = np.zeros(17, np.float32)
    _check(lib().rts_camera(yaw, pitch, zoom, ratio, _fp(out)), "rts_camera")
    return {"front": out[0:3].copy(), "right": out[3:6].copy(), "up": out[6:9].copy(),
            "left_bottom_corner": out[9:12].copy(), "half_h": float(out[12]), "half_w": float(out[13])}


def cpu_rand_origins(seed: int, n: int) -> np.ndarray:
    """randOrigin_1..n after srand(seed) (main.cpp:190; glibc rand restated in librtscene)."""
    out = np.zeros(n, np.float32)
    _check(lib().rts_cpu_rand_origins(seed, n, _fp(out)), "rts_cpu_rand_origins")
    return out


def glibc_rand(seed: int, n: int) -> np.ndarray:
    """The first n glibc rand() values after srand(seed) (rts_glibc_rand)."""
    out = np.zeros(n, np.int32)
    _check(lib().rts_glibc_rand(seed, n, out.ctypes.data_as(C.POINTER(C.c_int))), "rts_glibc_rand")
    return out


def tri_filter(tri: np.ndarray):
    """Traversal records {p1, N.x} {R2, N.y} {R3, N.z} and the edge-filter margin (k1, k0) of the
    HIP path (csrc/common/tri_filter.h) for tri = (n, 3, 4) float32 {p1, N.x} {p2, N.y} {p3, N.z}."""
    tri = np.ascontiguousarray(tri, np.float32)
    n = tri.shape[0]
    out = np.zeros_like(tri)
    k = (C.c_double * 2)()
    fl = np.zeros(1, np.int32)
    _check(lib().rts_tri_filter(_fp(tri), n, _fp(out), k, _ip(fl)), "rts_tri_filter")
    return out, float(k[0]), float(k[1]), int(fl[0])


def write_png(path: str, rgb: np.ndarray) -> None:
    """8-bit RGB (H, W, 3), row 0 = top -> PNG (rts_write_png, SaveFrame's stbi_write_png)."""
    a = np.ascontiguousarray(rgb, np.uint8)
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError("expected an (H, W, 3) uint8 image")
    _check(lib().rts_write_png(str(path).encode(), a.shape[1], a.shape[0], a.ctypes.data_as(C.POINTER(C.c_uint8))),
           "rts_write_png")
