"""ctypes bindings of librtamd.so (include/rt_abi.h): the MI355X path tracer.

``Renderer`` mirrors the reference's render-loop contract (src/sources/main.cpp:133-200):
static bindings (``set_scene``/``set_env``/``resize``) once, then per frame the uniform
list of main.cpp:181-199 (``FrameParams``) and a draw (``render``), with LoopNum handled as
main.cpp:175 does.  There is no CPU fallback: constructing a Renderer without a HIP device
raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes as C
import os
import dataclasses
from typing import Optional, Sequence

import numpy as np

from ._paths import lib_path

RT_OK, RT_ERR_ARG, RT_ERR_HIP, RT_ERR_STATE, RT_ERR_NOMEM, RT_ERR_NODEVICE, RT_ERR_LIMIT = 0, -1, -2, -3, -4, -5, -6
RT_MAX_FRAMES_PER_LAUNCH = 1024
RT_FLAG_NO_CULL = 1
RT_FLAG_COUNT_VISITS = 2
RT_FLAG_MEGAKERNEL = 4
RT_FLAG_NO_FINISH = 8
RT_FLAG_FINISH = 16
RT_FLAG_SERIAL = 32
RT_FLAG_SORTED_TRAVERSAL = 64
RT_ABI_VERSION = 6
RT_GATHER_AUTO, RT_GATHER_RCCL, RT_GATHER_PEER = 0, 1, 2
RT_LAYOUT_FRAME, RT_LAYOUT_LOCAL_TILES = 0, 1

_f32p = C.POINTER(C.c_float)
_i32p = C.POINTER(C.c_int32)

# every symbol include/rt_abi.h declares (tests check the library exports them all)
ABI_SYMBOLS = (
    "rt_create", "rt_destroy", "rt_last_error", "rt_device_info", "rt_set_scene", "rt_set_scene_encoded",
    "rt_update_materials", "rt_set_env", "rt_resize", "rt_reset", "rt_set_loop_num", "rt_get_loop_num",
    "rt_clear_accum", "rt_render_async", "rt_render", "rt_synchronize", "rt_stats_get", "rt_stats_reset",
    "rt_get_stream", "rt_set_stream", "rt_read_accum", "rt_write_accum", "rt_accum_device", "rt_copy_accum_device",
    "rt_assemble_frame", "rt_tonemap", "rt_set_max_paths", "rt_gather", "rt_set_tile_owners", "rt_get_tile_owners",
    "rt_tile_costs", "rt_set_finish", "rt_order_work", "rt_set_pipeline",
    "rt_tonemap_async", "rt_display_fetch", "rt_stats_get_sized", "rt_abi_version", "rt_gather_ex",
    "rt_gather_last_transport",
)
RT_DISPLAY_TONEMAP, RT_DISPLAY_GAMMA = 1, 2


class RtMaterial(C.Structure):
    _fields_ = [("v", C.c_float * 24)]


class RtSceneSoa(C.Structure):
    _fields_ = [
        ("n_triangles", C.c_int32),
        ("p1", _f32p), ("p2", _f32p), ("p3", _f32p),
        ("n1", _f32p), ("n2", _f32p), ("n3", _f32p),
        ("material_id", _i32p),
        ("materials", C.POINTER(RtMaterial)),
        ("n_materials", C.c_int32),
        ("n_nodes", C.c_int32),
        ("node_left", _i32p), ("node_right", _i32p), ("node_n", _i32p), ("node_index", _i32p),
        ("node_aa", _f32p), ("node_bb", _f32p),
    ]


class RtTiling(C.Structure):
    _fields_ = [("tile_w", C.c_int32), ("tile_h", C.c_int32), ("rank", C.c_int32), ("world", C.c_int32)]


class RtFrameParams(C.Structure):
    _fields_ = [
        ("position", C.c_float * 3), ("front", C.c_float * 3), ("right", C.c_float * 3), ("up", C.c_float * 3),
        ("left_bottom_corner", C.c_float * 3),
        ("half_h", C.c_float), ("half_w", C.c_float),
        ("enable_mis", C.c_int32), ("enable_env_map", C.c_int32), ("enable_bsdf", C.c_int32),
        ("env_intensity", C.c_float), ("env_angle", C.c_float),
        ("max_bounce", C.c_int32), ("max_iterations", C.c_int32),
        ("flags", C.c_int32),
    ]


class RtStats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("samples", C.c_uint64), ("internal_pops", C.c_uint64),
                ("leaf_pops", C.c_uint64), ("tri_tests", C.c_uint64), ("launches", C.c_uint64),
                ("kernel_ms", C.c_double), ("trace_launches", C.c_uint64), ("trace_ms", C.c_double),
                ("trace_iters", C.c_uint64), ("trace_iters_max", C.c_uint64), ("path_steps", C.c_uint64),
                ("p1_rays", C.c_uint64),
                # ABI 4
                ("pass0_steps", C.c_uint64), ("pass1_steps", C.c_uint64), ("finish_steps", C.c_uint64),
                ("trace_busy_ms", C.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


@dataclasses.dataclass
class FrameParams:
    """The per-frame uniforms of main.cpp:181-199 (RenderSettings.h:81-90 defaults)."""
    position: Sequence[float]
    front: Sequence[float]
    right: Sequence[float]
    up: Sequence[float]
    left_bottom_corner: Sequence[float]
    half_h: float
    half_w: float
    enable_mis: bool = True
    enable_env_map: bool = True
    enable_bsdf: bool = True
    env_intensity: float = 1.0
    env_angle: float = 0.0
    max_bounce: int = 8
    max_iterations: int = -1
    flags: int = 0

    def to_c(self) -> RtFrameParams:
        p = RtFrameParams()
        for k in ("position", "front", "right", "up", "left_bottom_corner"):
            arr = getattr(p, k)
            for i in range(3):
                arr[i] = float(np.float32(getattr(self, k)[i]))
        p.half_h, p.half_w = float(np.float32(self.half_h)), float(np.float32(self.half_w))
        p.enable_mis, p.enable_env_map, p.enable_bsdf = int(self.enable_mis), int(self.enable_env_map), int(self.enable_bsdf)
        p.env_intensity, p.env_angle = float(np.float32(self.env_intensity)), float(np.float32(self.env_angle))
        p.max_bounce, p.max_iterations, p.flags = int(self.max_bounce), int(self.max_iterations), int(self.flags)
        return p


_lib = None
_variants: dict = {}


def _share_torch_hip_runtime() -> None:
    """PyTorch-ROCm ships its own libamdhip64.so with the system's soname (libamdhip64.so.7);
    whichever is loaded first serves the whole process, and torch cannot run on the system one.
    Loading torch first makes librtamd.so bind to torch's runtime, so device pointers can be
    exchanged with torch tensors (bench.py's RCCL gather) in either import order."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def lib(path: Optional[str] = None) -> C.CDLL:
    """librtamd.so (or RTAMD_LIB, or an explicit build variant: each path is loaded once, with
    RTLD_LOCAL, so development variants can coexist in one process for A/B timing)."""
    global _lib
    _share_torch_hip_runtime()  # before the first librtamd load (see above)
    if path is not None:
        path = str(path)
        if path not in _variants:
            _variants[path] = _bind(C.CDLL(path))
        return _variants[path]
    if _lib is None:
        _lib = _bind(C.CDLL(os.environ.get("RTAMD_LIB") or str(lib_path("librtamd.so"))))
    return _lib


def dev_lib_path() -> str:
    """lib/librtamd_dev.so: the same kernels built with -DRT_DEV, whose development settings
    (test-only switches such as RT_CULL_EPS_SCALE, traversal-structure variants, A/B parameters)
    are read from the environment.  Tests that exercise those load it explicitly; the release
    librtamd.so reads no environment variable."""
    return str(lib_path("librtamd_dev.so"))


def _bind(L: C.CDLL) -> C.CDLL:
    vp = C.c_void_p
    L.rt_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.rt_destroy.argtypes = [vp]
    L.rt_last_error.argtypes = [vp]
    L.rt_last_error.restype = C.c_char_p
    L.rt_device_info.argtypes = [vp, _i32p, _i32p, _i32p]
    L.rt_set_scene.argtypes = [vp, C.POINTER(RtSceneSoa)]
    L.rt_set_scene_encoded.argtypes = [vp, _f32p, C.c_int32, _f32p, C.c_int32]
    L.rt_update_materials.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(RtMaterial)]
    L.rt_set_env.argtypes = [vp, _f32p, _f32p, C.c_int32, C.c_int32, C.c_int32]
    L.rt_resize.argtypes = [vp, C.c_int32, C.c_int32, C.POINTER(RtTiling)]
    L.rt_reset.argtypes = [vp]
    L.rt_set_loop_num.argtypes = [vp, C.c_int32]
    L.rt_get_loop_num.argtypes = [vp, _i32p]
    L.rt_clear_accum.argtypes = [vp]
    L.rt_render_async.argtypes = [vp, C.POINTER(RtFrameParams), _f32p, C.c_int32]
    L.rt_render.argtypes = [vp, C.POINTER(RtFrameParams), _f32p, C.c_int32, C.POINTER(RtStats)]
    L.rt_synchronize.argtypes = [vp]
    L.rt_stats_get.argtypes = [vp, C.POINTER(RtStats)]
    if hasattr(L, "rt_stats_get_sized"):  # ABI >= 4 (older builds are loaded for A/B timing)
        L.rt_stats_get_sized.argtypes = [vp, C.POINTER(RtStats), C.c_size_t]
        L.rt_abi_version.argtypes = []
    L.rt_stats_reset.argtypes = [vp]
    L.rt_get_stream.argtypes = [vp, C.POINTER(vp)]
    L.rt_set_stream.argtypes = [vp, vp]
    L.rt_read_accum.argtypes = [vp, _f32p, C.c_int32]
    L.rt_write_accum.argtypes = [vp, _f32p, C.c_int32]
    L.rt_accum_device.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_size_t), _i32p, _i32p]
    L.rt_copy_accum_device.argtypes = [vp, vp, C.c_size_t]
    L.rt_assemble_frame.argtypes = [vp, vp, C.c_int32, vp]
    L.rt_tonemap.argtypes = [vp, vp, C.c_int32, C.POINTER(C.c_uint8)]
    L.rt_set_max_paths.argtypes = [vp, C.c_uint64]
    if hasattr(L, "rt_set_finish"):  # (absent from older builds loaded for A/B timing)
        L.rt_set_finish.argtypes = [vp, C.c_int32, C.c_uint64]
    if hasattr(L, "rt_order_work"):
        L.rt_order_work.argtypes = [vp, C.POINTER(RtFrameParams), _f32p, C.c_int32]
    if hasattr(L, "rt_set_pipeline"):
        L.rt_set_pipeline.argtypes = [vp, C.c_int32]
        L.rt_tonemap_async.argtypes = [vp, vp, C.c_int32, C.c_int32]
        L.rt_display_fetch.argtypes = [vp, C.c_int32, C.POINTER(C.c_uint8)]
    L.rt_set_tile_owners.argtypes = [vp, _i32p, C.c_int32]
    L.rt_get_tile_owners.argtypes = [vp, _i32p, C.c_int32]
    L.rt_tile_costs.argtypes = [vp, C.POINTER(RtFrameParams), _f32p, C.c_int32, C.POINTER(C.c_uint64)]
    L.rt_gather.argtypes = [C.POINTER(vp), C.c_int32, _f32p]
    if hasattr(L, "rt_gather_ex"):
        L.rt_gather_ex.argtypes = [C.POINTER(vp), C.c_int32, _f32p, C.c_int32]
        L.rt_gather_last_transport.argtypes = [vp]
    return L


def _fp(a):
    return a.ctypes.data_as(_f32p)


def _ip(a):
    return a.ctypes.data_as(_i32p)


class Renderer:
    """One HIP device's path tracer (one per rank in multi-GPU runs)."""

    def __init__(self, device: int = 0, lib_path: Optional[str] = None):
        self._L = lib(lib_path)
        h = C.c_void_p()
        rc = self._L.rt_create(int(device), C.byref(h))
        if rc != RT_OK:
            raise RuntimeError(f"rt_create(device={device}) failed with {rc}: no usable HIP device "
                               "(librtamd has no CPU fallback)")
        self._h = h
        self.width = self.height = 0
        self.tiling = (32, 32, 0, 1)

    # ---------------------------------------------------------------- plumbing
    def _check(self, rc: int, what: str) -> None:
        if rc != RT_OK:
            msg = self._L.rt_last_error(self._h).decode(errors="replace")
            raise RuntimeError(f"{what} failed ({rc}): {msg}")

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self._L.rt_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_info(self) -> dict:
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        self._check(self._L.rt_device_info(self._h, C.byref(a), C.byref(b), C.byref(c)), "rt_device_info")
        return {"n_cus": a.value, "blocks_per_cu": b.value, "lds_bytes_per_block": c.value}

    # ------------------------------------------------------------ static data
    def set_scene_soa(self, soa: dict, nodes: dict) -> None:
        """soa: rts_scene_export_soa() arrays; nodes: rts_scene_nodes() arrays (reference numbering)."""
        keep = {k: np.ascontiguousarray(soa[k], np.float32) for k in ("p1", "p2", "p3", "n1", "n2", "n3")}
        mid = np.ascontiguousarray(soa["material_id"], np.int32)
        mats_np = np.ascontiguousarray(soa["materials"], np.float32).reshape(-1, 24)
        mats = (RtMaterial * max(1, len(mats_np)))()
        for i, row in enumerate(mats_np):
            for k in range(24):
                mats[i].v[k] = float(row[k])
        nd = {k: np.ascontiguousarray(nodes[k], np.int32) for k in ("left", "right", "n", "index")}
        aa = np.ascontiguousarray(nodes["aa"], np.float32)
        bb = np.ascontiguousarray(nodes["bb"], np.float32)
        s = RtSceneSoa()
        s.n_triangles = len(mid)
        s.p1, s.p2, s.p3 = _fp(keep["p1"]), _fp(keep["p2"]), _fp(keep["p3"])
        s.n1, s.n2, s.n3 = _fp(keep["n1"]), _fp(keep["n2"]), _fp(keep["n3"])
        s.material_id = _ip(mid)
        s.materials = mats
        s.n_materials = len(mats_np)
        s.n_nodes = len(nd["left"])
        s.node_left, s.node_right, s.node_n, s.node_index = (_ip(nd[k]) for k in ("left", "right", "n", "index"))
        s.node_aa, s.node_bb = _fp(aa), _fp(bb)
        self._check(self._L.rt_set_scene(self._h, C.byref(s)), "rt_set_scene")

    def set_scene_encoded(self, tri_enc: np.ndarray, node_enc: np.ndarray) -> None:
        t = np.ascontiguousarray(tri_enc, np.float32)
        n = np.ascontiguousarray(node_enc, np.float32)
        self._check(self._L.rt_set_scene_encoded(self._h, _fp(t), t.shape[0], _fp(n), n.shape[0]),
                    "rt_set_scene_encoded")

    def update_materials(self, first: int, count: int, material_texels: np.ndarray) -> None:
        m = RtMaterial()
        for k, v in enumerate(np.asarray(material_texels, np.float32).reshape(24)):
            m.v[k] = float(v)
        self._check(self._L.rt_update_materials(self._h, first, count, C.byref(m)), "rt_update_materials")

    def set_env(self, hdr: np.ndarray, cache: np.ndarray, hdr_resolution: Optional[int] = None) -> None:
        a = np.ascontiguousarray(hdr, np.float32)
        b = np.ascontiguousarray(cache, np.float32)
        h, w, _ = a.shape
        res = w if hdr_resolution is None else hdr_resolution
        self._check(self._L.rt_set_env(self._h, _fp(a), _fp(b), w, h, res), "rt_set_env")

    def resize(self, width: int, height: int, tile: int = 32, rank: int = 0, world: int = 1) -> None:
        t = RtTiling(tile, tile, rank, world)
        self._check(self._L.rt_resize(self._h, width, height, C.byref(t)), "rt_resize")
        self.width, self.height = width, height
        self.tiling = (tile, tile, rank, world)

    def set_tile_owners(self, owner: Sequence[int]) -> None:
        """owner[t] = rank rendering global tile t (rt_set_tile_owners; every rank sets the same map)."""
        o = np.ascontiguousarray(owner, np.int32)
        self._check(self._L.rt_set_tile_owners(self._h, o.ctypes.data_as(_i32p), len(o)), "rt_set_tile_owners")

    def tile_owners(self) -> np.ndarray:
        tx = (self.width + self.tiling[0] - 1) // self.tiling[0]
        ty = (self.height + self.tiling[1] - 1) // self.tiling[1]
        o = np.zeros(tx * ty, np.int32)
        self._check(self._L.rt_get_tile_owners(self._h, o.ctypes.data_as(_i32p), len(o)), "rt_get_tile_owners")
        return o

    def tile_costs(self, params: FrameParams, rand_origins: Sequence[float]) -> np.ndarray:
        """Per local tile cost of rendering these frames (rt_tile_costs; state left unchanged)."""
        ro = np.ascontiguousarray(rand_origins, np.float32)
        p = params.to_c()
        n = self.accum_device()["local_tiles"]
        out = np.zeros(max(1, n), np.uint64)
        self._check(self._L.rt_tile_costs(self._h, C.byref(p), _fp(ro), len(ro),
                                          out.ctypes.data_as(C.POINTER(C.c_uint64))), "rt_tile_costs")
        return out[:n]

    def order_work(self, params: FrameParams, rand_origins: Sequence[float]) -> None:
        """rt_order_work: probe these frames' per-block costs and queue the costliest 64-pixel
        blocks first (results unchanged; rt_resize restores the natural order)."""
        ro = np.ascontiguousarray(rand_origins, np.float32)
        p = params.to_c()
        self._check(self._L.rt_order_work(self._h, C.byref(p), _fp(ro), len(ro)), "rt_order_work")

    # ------------------------------------------------------------------ frames
    def reset(self) -> None:
        self._check(self._L.rt_reset(self._h), "rt_reset")

    def set_loop_num(self, n: int) -> None:
        self._check(self._L.rt_set_loop_num(self._h, n), "rt_set_loop_num")

    @property
    def loop_num(self) -> int:
        v = C.c_int32()
        self._check(self._L.rt_get_loop_num(self._h, C.byref(v)), "rt_get_loop_num")
        return v.value

    def set_max_paths(self, slots: int) -> None:
        """Path-state budget in pixel-frames (0: the library default); see rt_abi.h."""
        self._check(self._L.rt_set_max_paths(self._h, int(slots)), "rt_set_max_paths")

    def set_finish(self, pass_: int, max_slots: int) -> None:
        """rt_set_finish: end paths in the path-persistent finisher after pass `pass_ - 1` for frame
        groups of at most `max_slots` path slots (pass_ 0: never)."""
        self._check(self._L.rt_set_finish(self._h, int(pass_), int(max_slots)), "rt_set_finish")

    def set_pipeline(self, depth: int) -> None:
        """rt_set_pipeline: frames in flight across one-frame calls (1: off; results unchanged)."""
        self._check(self._L.rt_set_pipeline(self._h, int(depth)), "rt_set_pipeline")

    def clear_accum(self) -> None:
        self._check(self._L.rt_clear_accum(self._h), "rt_clear_accum")

    def render_async(self, params: FrameParams, rand_origins: Sequence[float]) -> None:
        ro = np.ascontiguousarray(rand_origins, np.float32)
        p = params.to_c()
        self._check(self._L.rt_render_async(self._h, C.byref(p), _fp(ro), len(ro)), "rt_render_async")

    def render(self, params: FrameParams, rand_origins: Sequence[float]) -> dict:
        ro = np.ascontiguousarray(rand_origins, np.float32)
        p = params.to_c()
        self._check(self._L.rt_render(self._h, C.byref(p), _fp(ro), len(ro), None), "rt_render")
        return self.stats()  # rt_render's own snapshot holds only the ABI-3 fields

    def synchronize(self) -> None:
        self._check(self._L.rt_synchronize(self._h), "rt_synchronize")

    def stats(self) -> dict:
        st = RtStats()  # zero-filled: a pre-ABI-4 build leaves the newer fields 0
        if hasattr(self._L, "rt_stats_get_sized"):
            self._check(self._L.rt_stats_get_sized(self._h, C.byref(st), C.sizeof(st)), "rt_stats_get_sized")
        else:
            self._check(self._L.rt_stats_get(self._h, C.byref(st)), "rt_stats_get")
        return st.as_dict()

    def reset_stats(self) -> None:
        self._check(self._L.rt_stats_reset(self._h), "rt_stats_reset")

    @property
    def stream(self) -> int:
        s = C.c_void_p()
        self._check(self._L.rt_get_stream(self._h, C.byref(s)), "rt_get_stream")
        return s.value or 0

    def set_stream(self, stream_ptr: Optional[int]) -> None:
        self._check(self._L.rt_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None), "rt_set_stream")

    # ----------------------------------------------------------- accumulation
    def read_accum(self) -> np.ndarray:
        """(H, W, 3) float32, row 0 = bottom row (GL framebuffer order); other ranks' pixels are 0."""
        out = np.zeros((self.height, self.width, 3), np.float32)
        self._check(self._L.rt_read_accum(self._h, _fp(out), RT_LAYOUT_FRAME), "rt_read_accum")
        return out

    def write_accum(self, img: np.ndarray) -> None:
        a = np.ascontiguousarray(img, np.float32)
        self._check(self._L.rt_write_accum(self._h, _fp(a), RT_LAYOUT_FRAME), "rt_write_accum")

    def accum_device(self) -> dict:
        p, n = C.c_void_p(), C.c_size_t()
        lt, mlt = C.c_int32(), C.c_int32()
        self._check(self._L.rt_accum_device(self._h, C.byref(p), C.byref(n), C.byref(lt), C.byref(mlt)),
                    "rt_accum_device")
        return {"ptr": p.value, "bytes": n.value, "local_tiles": lt.value, "max_local_tiles": mlt.value}

    def copy_accum_device(self, dst_ptr: int, nbytes: int) -> None:
        self._check(self._L.rt_copy_accum_device(self._h, C.c_void_p(dst_ptr), nbytes), "rt_copy_accum_device")

    def assemble_frame(self, gathered_ptr: int, world: int, frame_ptr: int) -> None:
        self._check(self._L.rt_assemble_frame(self._h, C.c_void_p(gathered_ptr), world, C.c_void_p(frame_ptr)),
                    "rt_assemble_frame")

    @staticmethod
    def gather(ranks: Sequence["Renderer"], transport: Optional[int] = None) -> np.ndarray:
        """rt_gather: the full (H, W, 3) frame (row 0 = bottom) from contexts ranks[r] = rank r of
        len(ranks), assembled on ranks[0]'s device (single-process multi-GPU); RCCL
        when every context has its own device, else peer copies (transport: rt_gather_ex's choice)."""
        r0 = ranks[0]
        hs = (C.c_void_p * len(ranks))(*[r._h.value for r in ranks])
        out = np.zeros((r0.height, r0.width, 3), np.float32)
        if transport is None:
            r0._check(r0._L.rt_gather(hs, len(ranks), _fp(out)), "rt_gather")
        else:
            r0._check(r0._L.rt_gather_ex(hs, len(ranks), _fp(out), int(transport)), "rt_gather_ex")
        return out

    def gather_transport(self) -> int:
        """the transport of this context's last gather as rank 0 (RT_GATHER_RCCL / RT_GATHER_PEER)"""
        return int(self._L.rt_gather_last_transport(self._h))

    def tonemap(self, flags: int = RT_DISPLAY_TONEMAP | RT_DISPLAY_GAMMA, frame_ptr: Optional[int] = None) -> np.ndarray:
        """The displayed 8-bit image (H, W, 3), row 0 = top: the tone-mapping pass / screen blit +
        SaveFrame's read-back (rt_abi.h rt_tonemap); frame_ptr = an assembled device frame."""
        out = np.zeros((self.height, self.width, 3), np.uint8)
        self._check(self._L.rt_tonemap(self._h, C.c_void_p(frame_ptr) if frame_ptr else None, int(flags),
                                       out.ctypes.data_as(C.POINTER(C.c_uint8))), "rt_tonemap")
        return out

    def tonemap_async(self, slot: int, flags: int = RT_DISPLAY_TONEMAP | RT_DISPLAY_GAMMA,
                      frame_ptr: Optional[int] = None) -> None:
        """Enqueue the display pass and its read-back into pinned slot `slot` (rt_tonemap_async)."""
        self._check(self._L.rt_tonemap_async(self._h, C.c_void_p(frame_ptr) if frame_ptr else None, int(flags),
                                             int(slot)), "rt_tonemap_async")
        self._disp_shape = {**getattr(self, "_disp_shape", {}), int(slot): (self.height, self.width)}

    def display_fetch(self, slot: int) -> np.ndarray:
        """Wait for slot `slot`'s display pass and return its 8-bit image (rt_display_fetch)."""
        h, w = getattr(self, "_disp_shape", {}).get(int(slot), (self.height, self.width))
        out = np.zeros((h, w, 3), np.uint8)
        self._check(self._L.rt_display_fetch(self._h, int(slot), out.ctypes.data_as(C.POINTER(C.c_uint8))),
                    "rt_display_fetch")
        return out
