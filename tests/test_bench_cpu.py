"""bench.py contract on CPU: randOrigin for any frame count (the driver's --steps 20 --warmup 5
needs 25,601+ frames), the in-tree glibc rand() restatement against the libc and the committed
fixture, and the self-launching multi-rank path in its gloo dry-run mode."""
import ctypes
import ctypes.util
import json
import subprocess
import sys
import time

import numpy as np
import pytest

from conftest import ROOT
from rtamd import configs as cf
from rtamd import scene_lib as sl


def test_rand_origins_cover_the_driver_bench():
    n = (5 + 20) * 1024 + 1 + 64
    ro = cf.rand_origins(n)
    assert ro.shape == (n,) and ro.dtype == np.float32
    fix = cf._fixture_bits()
    assert np.array_equal(ro[:len(fix)].view(np.uint32), fix)
    assert np.all((ro >= 674764.0) & (ro <= 2 * 674764.0))
    assert np.array_equal(cf.rand_origins(100, offset=20000), ro[20000:20100])
    assert np.array_equal(cf.rand_origins(10, offset=16380), ro[16380:16390])  # straddles the fixture end


def _libc():
    name = ctypes.util.find_library("c")
    if not name:
        return None
    L = ctypes.CDLL(name)
    try:
        L.gnu_get_libc_version.restype = ctypes.c_char_p
        L.gnu_get_libc_version()
    except AttributeError:
        return None  # not glibc: its rand() is another generator
    return L


@pytest.mark.parametrize("seed", [0, 1, 20221002, 123456789, 2**31 - 1, 2**32 - 1])
def test_glibc_rand_restatement_equals_libc(seed):
    L = _libc()
    if L is None:
        pytest.skip("host libc is not glibc")
    L.srand(ctypes.c_uint(seed))
    want = np.array([L.rand() for _ in range(5000)], np.int32)
    assert np.array_equal(sl.glibc_rand(seed, 5000), want)


def _bench(*args, timeout=240):
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_dry_run_driver_arguments():
    d = _bench("--gpus", "1", "--steps", "20", "--warmup", "5", "--dry-run")
    assert d["dry_run"] and d["n_gpus"] == 1
    assert d["frames_planned"] == (5 + 20) * 1024 + 1 + 64
    assert d["pixels_covered"] == d["frame_pixels"] == 1920 * 1080


def test_bench_self_launches_two_gloo_ranks():
    d = _bench("--gpus", "2", "--steps", "20", "--warmup", "5", "--dry-run")
    assert d["n_gpus"] == 2 and d["gather_ok"]
    assert d["pixels_covered"] == 1920 * 1080


def test_bench_launcher_stops_the_other_ranks_when_one_fails():
    """A rank that exits early would leave the others waiting in the rendezvous; the launcher
    stops them and returns the failing rank's status instead of hanging."""
    t0 = time.time()
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run", "--fail-rank", "1"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert not any(ln.startswith("{") for ln in p.stdout.splitlines())
    assert time.time() - t0 < 90
