"""The C-ABI libraries load and export every symbol their headers declare (no GPU calls)."""
import ctypes as C
import re

import pytest

from conftest import ROOT
from rtamd import renderer, scene_lib


def _declared(header):
    text = (ROOT / "include" / header).read_text()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+(rt[s]?_\w+)\s*\(", text, re.M)))


@pytest.mark.parametrize("header,libname", [("rt_abi.h", "librtamd.so"), ("rt_abi.h", "librtamd_dev.so"),
                                            ("rt_scene.h", "librtscene.so")])
def test_library_exports_every_declared_symbol(header, libname):
    syms = _declared(header)
    assert len(syms) > 10
    lib = C.CDLL(str(ROOT / "opengl-ray-tracing-framework_amd" / "lib" / libname))
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_abi():
    assert sorted(renderer.ABI_SYMBOLS) == _declared("rt_abi.h")


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(RuntimeError, match="no usable HIP device"):
        renderer.Renderer(0)


def test_scene_lib_error_codes():
    with pytest.raises(RuntimeError):
        scene_lib.Mesh.load("/nonexistent.obj")
    with pytest.raises(RuntimeError):
        scene_lib.load_hdr("/nonexistent.hdr")


def test_release_library_reads_no_environment():
    """Development settings (rt_render.hip knob(): RT_CULL_EPS_SCALE, RT_BVH_WIDTH, RT_GROUPS, ...)
    exist only in lib/librtamd_dev.so (-DRT_DEV): the release library neither imports getenv nor
    carries any of their names, so no process environment can change what it renders."""
    libdir = ROOT / "opengl-ray-tracing-framework_amd" / "lib"
    rel = (libdir / "librtamd.so").read_bytes()
    dev = (libdir / "librtamd_dev.so").read_bytes()
    assert b"getenv" not in rel
    assert b"RT_CULL_EPS_SCALE" not in rel and b"RT_BVH_WIDTH" not in rel
    assert b"RT_CULL_EPS_SCALE" in dev and b"getenv" in dev


def test_stats_struct_matches_header(tmp_path):
    """The ctypes rt_stats mirrors include/rt_abi.h field for field (offsets and size from gcc on the
    header itself), and rt_abi_version() (no device needed) is the header's RT_ABI_VERSION."""
    fields = [f for f, _ in renderer.RtStats._fields_]
    src = tmp_path / "probe.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "rt_abi.h"\nint main(void) {\n'
                   '  printf("%zu %d\\n", sizeof(rt_stats), RT_ABI_VERSION);\n' +
                   "".join(f'  printf("%zu\\n", offsetof(rt_stats, {f}));\n' for f in fields) + "  return 0;\n}\n")
    import subprocess
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", str(ROOT / "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    size, ver = int(out[0]), int(out[1])
    assert size == C.sizeof(renderer.RtStats)
    assert [int(x) for x in out[2:]] == [getattr(renderer.RtStats, f).offset for f in fields]
    assert ver == renderer.RT_ABI_VERSION
    lib = C.CDLL(str(ROOT / "opengl-ray-tracing-framework_amd" / "lib" / "librtamd.so"))
    assert lib.rt_abi_version() == ver


def test_flag_constants_match_header():
    """Every RT_FLAG_* of include/rt_abi.h has the same value in the ctypes binding (and no
    binding flag is missing from the header)."""
    text = (ROOT / "include" / "rt_abi.h").read_text()
    header = {k: int(v) for k, v in re.findall(r"^\s*(RT_FLAG_\w+)\s*=\s*(\d+)", text, re.M)}
    binding = {k: getattr(renderer, k) for k in dir(renderer) if k.startswith("RT_FLAG_")}
    assert len(header) >= 7
    assert header == binding


C_BIN = ROOT / "tests" / "c" / "bin" / "abi_stats"


def test_c_binding_builds_against_the_header():
    """tests/c/abi_stats.c (built by __graft_entry__.build() with gcc) links librtamd.so the way a
    C caller of include/rt_abi.h does; without a GPU it must fail cleanly in rt_create."""
    import subprocess
    import torch
    assert C_BIN.exists(), "make -C tests/c"
    if torch.cuda.is_available():
        pytest.skip("a GPU is present: tests/test_abi.py::test_c_binding_reads_the_abi4_tail runs it")
    p = subprocess.run([str(C_BIN)], capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and "rt_create" in p.stderr, (p.returncode, p.stderr)


@pytest.mark.gpu
def test_c_binding_reads_the_abi4_tail():
    """a C caller compiled against this header gets the ABI-4 fields of rt_stats through
    rt_stats_get_sized, and rt_stats_get writes only the ABI-3 prefix (tests/c/abi_stats.c)."""
    import subprocess
    p = subprocess.run([str(C_BIN)], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "abi_stats ok" in p.stdout
