#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh output directory into profiles/.

    python3 tools/summarize_profile.py <dir> <tag> '<workload json>'

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats), profiles/<tag>_summary.json (per
kernel: launches, average duration, PMC counters per launch) and, for the bench's dominant
kernel, profiles/pmc_<config>.json that bench.py reads when its workload key matches.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE is doubled per
MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B read requests at 64 B; that correction is
calibrated on wide coalesced streams, so for gathers the absolute value is indicative).
Effective clock = GRBM_GUI_ACTIVE / 8 (summed over the XCDs) / duration (same guide, DVFS).
Counters are taken from the timed bench launches (wf_*<false, ...>; the visit-counting frame
runs the <true, ...> instantiation and is excluded).
"""
import csv
import json
import shutil
import statistics
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1])
tag = sys.argv[2]
cfg = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}
dst = Path(__file__).resolve().parent.parent / "profiles"
dst.mkdir(exist_ok=True)
KERNELS = {"wf_trace": "wf_trace<false", "wf_shade": "wf_shade<", "wf_blend": "wf_blend", "wf_camera": "wf_camera"}


def kname(full):
    for k, pat in KERNELS.items():
        if pat in full:
            return k
    return None


shutil.copyfile(src / "trace" / "run_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
durs, regs = defaultdict(list), {}
for r in csv.DictReader(open(src / "trace" / "run_kernel_trace.csv")):
    k = kname(r["Kernel_Name"])
    if k:
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        regs[k] = {"vgpr": int(r.get("Arch_VGPR_Count", r.get("VGPR_Count", 0)) or 0),
                   "sgpr": int(r.get("SGPR_Count", 0) or 0), "lds": int(r.get("LDS_Block_Size", 0) or 0),
                   "scratch": int(r.get("Scratch_Size", 0) or 0)}


def counters(name):
    """per kernel: counter -> mean over launches (and the durations seen in that pass)"""
    out = defaultdict(lambda: defaultdict(list))
    p = src / name / "run_counter_collection.csv"
    if not p.exists():
        return {}
    for r in csv.DictReader(open(p)):
        k = kname(r["Kernel_Name"])
        if k:
            out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: statistics.mean(v) for c, v in d.items()} for k, d in out.items()}


passes = [counters(n) for n in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2", "pmc_tcc")]
summary = {"workload": cfg, "kernels": {}}
for k in KERNELS:
    if not durs.get(k):
        continue
    c = {}
    for p in passes:
        c.update(p.get(k, {}))
    ms = statistics.mean(durs[k])
    e = {"launches_traced": len(durs[k]), "avg_launch_ms": round(ms, 4), "total_ms": round(sum(durs[k]), 2),
         **regs[k], "counters_per_launch": {n: round(v, 1) for n, v in sorted(c.items())}}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        e["hbm_bytes_per_launch"] = round((2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024)
        e["hbm_tbs"] = round(e["hbm_bytes_per_launch"] / (ms * 1e-3) / 1e12, 3)
    if c.get("GRBM_GUI_ACTIVE"):
        e["clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9, 3)
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
        e["valu_lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 4)
    if c.get("SQ_WAVE_CYCLES"):
        w = c["SQ_WAVE_CYCLES"]
        e["wave_cycle_split"] = {"waiting": round(c.get("SQ_WAIT_ANY", 0) / w, 3),
                                 "issue_stalled": round(c.get("SQ_WAIT_INST_ANY", 0) / w, 3),
                                 "issuing": round(c.get("SQ_ACTIVE_INST_ANY", 0) / w, 3)}
    if c.get("TCC_HIT_sum"):
        e["l2_hit"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    summary["kernels"][k] = e
tot = sum(v["total_ms"] for v in summary["kernels"].values())
for v in summary["kernels"].values():
    v["time_share"] = round(v["total_ms"] / tot, 4)
(dst / f"{tag}_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
if cfg.get("config") and "wf_trace" in summary["kernels"]:
    t = summary["kernels"]["wf_trace"]
    pm = {"kernel": "wf_trace", **cfg, "avg_launch_ms": t["avg_launch_ms"],
          "hbm_bytes_per_launch": t.get("hbm_bytes_per_launch"), "clock_ghz": t.get("clock_ghz"),
          "SQ": {n: v for n, v in t["counters_per_launch"].items() if n.startswith("SQ_")},
          "source": f"profiles/{tag}_summary.json"}
    (dst / f"pmc_{cfg['config']}.json").write_text(json.dumps(pm, indent=1) + "\n")
print(json.dumps(summary, indent=1))
