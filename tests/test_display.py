"""Display step: tone mapping pass / screen blit + 8-bit read-back + PNG.

CPU: the oracle's restatement of fragment_shader_tone_mapping.glsl:66-93 against an independent
numpy float32 evaluation of the same formulas, SaveFrame's vertical flip, and the PNG writer
(rts_write_png) decoded back with Python's zlib.  GPU: rt_tonemap against the oracle, bit for bit.
"""
import struct
import zlib

import numpy as np
import pytest

import oracle as orc
from helpers import frames_for, gpu_render, oracle_render
from rtamd import configs as cf
from rtamd import scene_lib as sl
from rtamd.renderer import RT_DISPLAY_GAMMA, RT_DISPLAY_TONEMAP


def _frame(seed=3, H=17, W=23):
    rng = np.random.default_rng(seed)
    f = (rng.random((H, W, 3), dtype=np.float32) * np.float32(4.0)).astype(np.float32)
    f[0, 0] = [0.0, 1e-30, 1e30]
    f[1, 1] = [np.nan, -1.0, 0.5]
    return f


def _aces_np(c):
    c = c.astype(np.float32)
    a, b, y, d, e = (np.float32(v) for v in (2.51, 0.03, 2.43, 0.59, 0.14))
    with np.errstate(invalid="ignore", over="ignore"):
        r = (c * (a * c + b)) / (c * (y * c + d) + e)
    return np.clip(np.nan_to_num(r, nan=0.0), 0, 1).astype(np.float32)  # fminf/fmaxf: NaN -> bound


def _unorm8(c):
    c = np.clip(np.nan_to_num(c.astype(np.float32), nan=0.0), 0, 1).astype(np.float32)
    return np.floor(c * np.float32(255.0) + np.float32(0.5)).astype(np.uint8)


def test_tonemap_matches_independent_float32_evaluation():
    f = _frame()
    out = orc.display(f, RT_DISPLAY_TONEMAP)
    ref = _unorm8(_aces_np(f))[::-1]
    assert np.array_equal(out, ref)


def test_blit_and_flip():
    f = _frame()
    out = orc.display(f, 0)  # enableToneMapping off: the screen shader draws the accumulation
    assert np.array_equal(out, _unorm8(f)[::-1])
    assert np.array_equal(out[0], _unorm8(f[-1]))  # SaveFrame: PNG row 0 = top = GL row H-1


def test_gamma_close_to_numpy_pow():
    f = _frame()
    out = orc.display(f, RT_DISPLAY_TONEMAP | RT_DISPLAY_GAMMA).astype(int)
    ref = _unorm8(np.power(_aces_np(f), np.float32(1.0 / 2.2)))[::-1].astype(int)
    assert np.abs(out - ref).max() <= 1  # glsl_math pow_ vs libm powf: ulp-level, 8-bit rounding
    assert (out == ref).mean() > 0.995


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        typ = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(typ + body) & 0xffffffff, typ
        chunks.setdefault(typ, b"")
        chunks[typ] += body
        pos += 12 + n
    w, h, depth, ctype = struct.unpack(">IIBB", chunks[b"IHDR"][:10])
    raw = zlib.decompress(chunks[b"IDAT"])
    rows = np.frombuffer(raw, np.uint8).reshape(h, 1 + 3 * w)
    assert (rows[:, 0] == 0).all() and depth == 8 and ctype == 2 and b"IEND" in chunks
    return rows[:, 1:].reshape(h, w, 3)


@pytest.mark.parametrize("shape", [(1, 1), (17, 23), (300, 250)])  # > 64 KiB: several stored blocks
def test_png_writer_round_trip(tmp_path, shape):
    rng = np.random.default_rng(shape[0])
    img = rng.integers(0, 256, (*shape, 3), dtype=np.uint8)
    p = tmp_path / "x.png"
    sl.write_png(str(p), img)
    assert np.array_equal(_read_png(p), img)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, RT_DISPLAY_TONEMAP, RT_DISPLAY_TONEMAP | RT_DISPLAY_GAMMA])
def test_gpu_tonemap_matches_oracle(gpu_renderer, env_maps, flags):
    sd = cf.config_scene("C3")
    W, H = 64, 36
    fp = cf.frame_params(W, H)
    ro, frames = frames_for(fp, 1, 2)
    ref, _ = oracle_render(sd, env_maps, W, H, frames)
    img, _ = gpu_render(gpu_renderer, sd, env_maps, W, H, fp, ro, tile=16)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    expect = orc.display(ref, flags)
    assert np.array_equal(gpu_renderer.tonemap(flags), expect)
    # the assembled-frame input (what rank 0 displays after the RCCL gather)
    import torch
    frame = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    torch.cuda.synchronize()
    assert np.array_equal(gpu_renderer.tonemap(flags, frame.data_ptr()), expect)
