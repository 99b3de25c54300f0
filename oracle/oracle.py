"""TEST INFRASTRUCTURE ONLY — ctypes binding of oracle/liboracle.so (oracle/rt_oracle.cpp).

The CPU restatement of src/shaders/fragment_shader_ray_tracing.glsl.  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as
the checker / the timed CPU baseline — never as a product path.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import os
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
_f32p = C.POINTER(C.c_float)


class OrcScene(C.Structure):
    _fields_ = [("triangles", _f32p), ("n_triangles", C.c_int), ("nodes", _f32p), ("n_nodes", C.c_int),
                ("hdr_map", _f32p), ("hdr_cache", _f32p), ("hdr_w", C.c_int), ("hdr_h", C.c_int),
                ("hdr_resolution", C.c_int)]


class OrcFrame(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("front", C.c_float * 3), ("right", C.c_float * 3),
                ("up", C.c_float * 3), ("left_bottom_corner", C.c_float * 3), ("half_h", C.c_float),
                ("half_w", C.c_float), ("loop_num", C.c_int), ("rand_origin", C.c_float),
                ("enable_mis", C.c_int), ("enable_env_map", C.c_int), ("enable_bsdf", C.c_int),
                ("env_intensity", C.c_float), ("env_angle", C.c_float), ("max_bounce", C.c_int),
                ("max_iterations", C.c_int)]


class OrcCounters(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("internal_pops", C.c_uint64), ("leaf_pops", C.c_uint64),
                ("tri_tests", C.c_uint64), ("closer_updates", C.c_uint64), ("samples", C.c_uint64),
                ("env_fetches", C.c_uint64), ("cache_fetches", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_libs: dict = {}


def lib(variant: str = "") -> C.CDLL:
    """liboracle.so, or liboracle_<variant>.so ("libm": the GLSL builtins from the C library's
    fp32 functions instead of glsl_math.h's polynomials)."""
    if variant not in _libs:
        p = ORACLE_DIR / (f"liboracle_{variant}.so" if variant else "liboracle.so")
        if not p.exists():
            raise FileNotFoundError(f"{p} not built: make -C {ORACLE_DIR}")
        L = C.CDLL(str(p))
        L.orc_render.argtypes = [C.POINTER(OrcScene), C.POINTER(OrcFrame), C.c_int, C.c_int, C.c_int, C.c_int,
                                 C.c_int, C.c_int, C.c_int, _f32p, C.POINTER(OrcCounters), C.c_int]
        L.orc_trace.argtypes = [C.POINTER(OrcScene), _f32p, _f32p, _f32p, _f32p, _f32p, C.POINTER(C.c_int)]
        L.orc_wang_rand.argtypes = [C.POINTER(C.c_uint32)]
        L.orc_wang_rand.restype = C.c_float
        L.orc_sobol.argtypes = [C.c_int, C.c_int]
        L.orc_sobol.restype = C.c_float
        L.orc_sobol_vec2.argtypes = [C.c_int, C.c_int, _f32p]
        L.orc_math.argtypes = [C.c_int, C.c_float, C.c_float]
        L.orc_math.restype = C.c_float
        L.orc_dielectric_fresnel.argtypes = [C.c_float, C.c_float]
        L.orc_dielectric_fresnel.restype = C.c_float
        L.orc_gtr2.argtypes = [C.c_float, C.c_float]
        L.orc_gtr2.restype = C.c_float
        L.orc_hdr_pdf.argtypes = [C.POINTER(OrcScene), _f32p, C.c_float]
        L.orc_hdr_pdf.restype = C.c_float
        L.orc_sample_hdr.argtypes = [C.POINTER(OrcScene), C.c_float, C.c_float, _f32p]
        L.orc_to_spherical.argtypes = [_f32p, C.c_float, _f32p]
        L.orc_disney_eval.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, _f32p]
        L.orc_disney_sample.argtypes = [_f32p, _f32p, _f32p, _f32p, _f32p, _f32p, _f32p, C.POINTER(C.c_int)]
        L.orc_display.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8)]
        _libs[variant] = L
    return _libs[variant]


def _fp(a: np.ndarray):
    return a.ctypes.data_as(_f32p)


class OracleScene:
    """Holds the arrays alive for an OrcScene (reference encodings + env textures)."""

    def __init__(self, tri_enc: np.ndarray, node_enc: np.ndarray, hdr: np.ndarray, cache: np.ndarray,
                 hdr_resolution: Optional[int] = None):
        self.tri = np.ascontiguousarray(tri_enc, np.float32)
        self.nodes = np.ascontiguousarray(node_enc, np.float32)
        self.hdr = np.ascontiguousarray(hdr, np.float32)
        self.cache = np.ascontiguousarray(cache, np.float32)
        h, w, _ = self.hdr.shape
        self.c = OrcScene(_fp(self.tri), self.tri.shape[0], _fp(self.nodes), self.nodes.shape[0],
                          _fp(self.hdr), _fp(self.cache), w, h, w if hdr_resolution is None else hdr_resolution)


def frame_struct(params: dict) -> OrcFrame:
    f = OrcFrame()
    for k in ("position", "front", "right", "up", "left_bottom_corner"):
        arr = getattr(f, k)
        for i in range(3):
            arr[i] = float(np.float32(params[k][i]))
    f.half_h, f.half_w = float(np.float32(params["half_h"])), float(np.float32(params["half_w"]))
    f.loop_num = int(params["loop_num"])
    f.rand_origin = float(np.float32(params["rand_origin"]))
    f.enable_mis, f.enable_env_map, f.enable_bsdf = (int(params[k]) for k in ("enable_mis", "enable_env_map",
                                                                              "enable_bsdf"))
    f.env_intensity, f.env_angle = float(np.float32(params["env_intensity"])), float(np.float32(params["env_angle"]))
    f.max_bounce, f.max_iterations = int(params["max_bounce"]), int(params["max_iterations"])
    return f


def render(scene: OracleScene, frames: Sequence[dict], W: int, H: int, x0: int = 0, y0: int = 0,
           w: Optional[int] = None, h: Optional[int] = None, accum: Optional[np.ndarray] = None,
           threads: int = 0, variant: str = ""):
    """Render len(frames) progressive frames over the sub-rect; returns (accum (h,w,3), counters)."""
    w = W - x0 if w is None else w
    h = H - y0 if h is None else h
    acc = np.zeros((h, w, 3), np.float32) if accum is None else np.ascontiguousarray(accum, np.float32).copy()
    fr = (OrcFrame * len(frames))(*[frame_struct(p) for p in frames])
    cnt = OrcCounters()
    rc = lib(variant).orc_render(C.byref(scene.c), fr, len(frames), W, H, x0, y0, w, h, _fp(acc), C.byref(cnt),
                          threads or (os.cpu_count() or 1))
    if rc != 0:
        raise RuntimeError(f"orc_render failed: {rc}")
    return acc, cnt.as_dict()


def display(frame: np.ndarray, flags: int = 3) -> np.ndarray:
    """Tone map / blit + 8-bit conversion + SaveFrame flip of an (H, W, 3) float frame (row 0 =
    bottom) -> (H, W, 3) uint8, row 0 = top (TM:66-93, Utility.h:19-30)."""
    f = np.ascontiguousarray(frame, np.float32)
    out = np.zeros(f.shape, np.uint8)
    lib().orc_display(f.ctypes.data_as(_f32p), f.shape[1], f.shape[0], int(flags), out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out
