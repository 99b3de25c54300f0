"""The multi-rank bench on one GPU (bench.py --rehearse): every rank renders its tile share on
device 0, the tile-cost balance and the frame-end gather run over gloo, rank 0 assembles the
frame.  The assembled frame must equal the one-rank frame bit for bit (pixels are
independent), so the N-rank path the driver's scaling run takes is checked on real hardware
except for the RCCL transport itself."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
COMMON = ["--steps", "1", "--warmup", "1", "--frames-per-step", "4", "--width", "256", "--height", "160",
          "--cpu-seconds", "0", "--single-frames", "0", "--frame-sha"]


def _bench(*args):
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), *COMMON, *args], capture_output=True, text=True,
                       timeout=300, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])


@pytest.mark.parametrize("n,extra", [(2, []), (3, ["--no-balance"]), (2, ["--pipeline-steps"])])
def test_multi_rank_bench_frame_equals_one_rank(n, extra):
    one = _bench("--gpus", "1")
    many = _bench("--gpus", str(n), "--rehearse", *extra)
    assert many["n_gpus"] == n and many["rehearsal"]
    assert many["frame_sha256"] == one["frame_sha256"]
    assert many["rays_per_sample"] == one["rays_per_sample"]
    # the line shows which collective backend saw how many ranks, and each rank's time
    co = many["collective"]
    assert co["backend"] == "gloo" and co["world"] == n and co["rehearsal"]
    assert len(co["rank_ms"]) == n and len(co["gather_ms_per_rank"]) == n and co["gather_ms"] >= 0
    assert co["rank_max_over_mean"] >= 1.0
    assert one["collective"]["world"] == 1 and one["collective"]["backend"] is None


def test_eight_rank_bench_at_full_size_frame_equals_one_rank():
    """The driver's largest configuration: 8 ranks of 1920x1080 tiles, cost-balanced map."""
    full = ["--width", "1920", "--height", "1080", "--frames-per-step", "2"]
    one = _bench("--gpus", "1", *full)
    eight = _bench("--gpus", "8", "--rehearse", *full)
    assert eight["frame_sha256"] == one["frame_sha256"]
    assert eight["rays_per_sample"] == one["rays_per_sample"]
