#!/usr/bin/env python3
"""Summarise a tools/profile_gpu.sh output directory into profiles/.

    python3 tools/summarize_profile.py <dir> <tag> '<workload json>'

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats), profiles/<tag>_summary.json (per
kernel: launches, average duration, PMC counters per launch) and, for the bench's dominant
kernel, profiles/pmc_<config>.json that bench.py reads when its workload key matches.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE is doubled per
MI355X_MICROARCH.md §HBM (gfx950 tallies 128-B read requests at 64 B; that correction is
calibrated on wide coalesced streams, so for gathers the absolute value is indicative).
Standalone duration = the mean launch duration in the PMC passes' own kernel traces (counter
collection serialises the dispatches); the trace pass's durations are the co-running ones.
Effective clock = GRBM_GUI_ACTIVE / 8 (summed over the XCDs) / the same pass's standalone
duration (same guide, DVFS), reported only for launches of >= 0.3 ms (shorter ones read high).
Launches are taken from the bench run up to its visit-counting frame: every dispatch from the first
wf_trace<true, ...> (the COUNT instantiation that frame runs) on is dropped, wf_shade's included
(its 18 near-empty launches had been averaged in).  probe_avg_launch_ms = the mean of the
last `probe_trace_launches` wf_trace launches before that frame in the trace pass: bench.py's
standalone probe (one frame group, RT_FLAG_SERIAL), the figure its roofline divides by.
A wf_trace "launch" is one bounce pass's traversal: with split queues (round 6) a secondary pass is
two dispatches, wf_trace<..., 2> (its shadow rays) then wf_trace<..., 1> (its continuations), so
wf_trace's durations and counters are summed over a pass's dispatches (an any-hit dispatch joins
the dispatch after it) and `dispatches` breaks the trace pass down per instantiation.
"""
import csv
import json
import re
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


def rows(path):
    """kernel-trace / counter rows of one pass, in dispatch order, up to the visit-count frame"""
    rs = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Dispatch_Id"]))
    cut = next((int(r["Dispatch_Id"]) for r in rs if "wf_trace<true" in r["Kernel_Name"]), None)
    return [r for r in rs if cut is None or int(r["Dispatch_Id"]) < cut]


def any_hit(full):
    """a wf_trace<..., 2> dispatch: the shadow-ray half of a split pass (joins the next dispatch)"""
    return re.search(r"wf_trace<[^>]*, 2>", full) is not None


def launch_key(k, r, state):
    """the launch a dispatch belongs to: its own Dispatch_Id, or for an any-hit wf_trace dispatch
    the next wf_trace dispatch's (state carries the pending ones)"""
    d = r["Dispatch_Id"]
    if k != "wf_trace":
        return d
    if any_hit(r["Kernel_Name"]):
        state.setdefault("pend", []).append(d)
        return None
    for p in state.pop("pend", []):
        state.setdefault("alias", {})[p] = d
    return d


shutil.copyfile(src / "trace" / "run_kernel_stats.csv", dst / f"{tag}_kernel_stats.csv")
durs, regs = defaultdict(list), {}
inst = defaultdict(list)  # wf_trace instantiation -> dispatch durations (trace pass)
carry = 0.0
for r in rows(src / "trace" / "run_kernel_trace.csv"):
    k = kname(r["Kernel_Name"])
    if k:
        ms_ = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        if k == "wf_trace":
            inst[r["Kernel_Name"].split("(")[0].replace("void rtd::", "")].append(ms_)
            if any_hit(r["Kernel_Name"]):
                carry += ms_
                continue
            ms_, carry = ms_ + carry, 0.0
        durs[k].append(ms_)
        regs[k] = {"vgpr": int(r.get("Arch_VGPR_Count", r.get("VGPR_Count", 0)) or 0),
                   "sgpr": int(r.get("SGPR_Count", 0) or 0), "lds": int(r.get("LDS_Block_Size", 0) or 0),
                   "scratch": int(r.get("Scratch_Size", 0) or 0)}


def standalone(name):
    """per kernel: (dispatch id -> duration ms) of a PMC pass's own kernel trace"""
    p = src / name / "run_kernel_trace.csv"
    out = defaultdict(dict)
    if p.exists():
        st, carry = {}, 0.0
        for r in rows(p):
            k = kname(r["Kernel_Name"])
            if k:
                ms_ = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                if launch_key(k, r, st) is None:
                    carry += ms_
                    continue
                out[k][r["Dispatch_Id"]] = ms_ + (carry if k == "wf_trace" else 0.0)
                if k == "wf_trace":
                    carry = 0.0
    return out


def counters(name):
    """per kernel: counter -> mean over launches (and the durations seen in that pass)"""
    out = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> counter -> launch -> value
    p = src / name / "run_counter_collection.csv"
    if not p.exists():
        return {}
    st = {}
    rs = rows(p)
    for r in rs:  # (a dispatch's counters come in several rows: resolve launches in dispatch order first)
        k = kname(r["Kernel_Name"])
        if k and r["Dispatch_Id"] not in st.setdefault("seen", set()):
            st["seen"].add(r["Dispatch_Id"])
            launch_key(k, r, st)
    alias = st.get("alias", {})
    for r in rs:
        k = kname(r["Kernel_Name"])
        if k:
            d = alias.get(r["Dispatch_Id"], r["Dispatch_Id"])
            out[k][r["Counter_Name"]][d] += float(r["Counter_Value"])
    return {k: {c: statistics.mean(v.values()) for c, v in d.items()} for k, d in out.items()}


PASSES = ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2", "pmc_tcc")
passes = [counters(n) for n in PASSES]
solo = {n: standalone(n) for n in PASSES}
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
    sd = [statistics.mean(solo[n][k].values()) for n in PASSES if solo[n].get(k)]
    if sd:
        e["avg_launch_ms_standalone"] = round(statistics.mean(sd), 4)
        e["avg_launch_ms_standalone_per_pass"] = [round(x, 4) for x in sd]
    g = solo["pmc_sq2"].get(k)
    if c.get("GRBM_GUI_ACTIVE") and g:
        gms = statistics.mean(g.values())
        if gms >= 0.3:
            e["effective_clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (gms * 1e-3) / 1e9, 3)
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
        e["valu_lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 4)
    if c.get("SQ_WAVE_CYCLES"):
        w = c["SQ_WAVE_CYCLES"]
        e["wave_cycle_split"] = {"waiting": round(c.get("SQ_WAIT_ANY", 0) / w, 3),
                                 "issue_stalled": round(c.get("SQ_WAIT_INST_ANY", 0) / w, 3),
                                 "issuing": round(c.get("SQ_ACTIVE_INST_ANY", 0) / w, 3)}
    npr = int(cfg.get("probe_trace_launches", 0))
    if k == "wf_trace" and npr and len(durs[k]) > npr:
        e["probe_avg_launch_ms"] = round(statistics.mean(durs[k][-npr:]), 4)
        e["probe_launches"] = npr
    if k == "wf_trace" and inst:
        e["dispatches"] = {n: {"count": len(v), "avg_ms": round(statistics.mean(v), 4), "total_ms": round(sum(v), 2)}
                           for n, v in inst.items()}
    if c.get("TCC_HIT_sum"):
        e["l2_hit"] = round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
    summary["kernels"][k] = e
tot = sum(v["total_ms"] for v in summary["kernels"].values())
for v in summary["kernels"].values():
    v["time_share"] = round(v["total_ms"] / tot, 4)
(dst / f"{tag}_summary.json").write_text(json.dumps(summary, indent=1) + "\n")
if cfg.get("config") and "wf_trace" in summary["kernels"]:
    pm = {**cfg, "kernels": {}, "source": f"profiles/{tag}_summary.json"}
    for k in ("wf_trace", "wf_shade"):
        t = summary["kernels"].get(k)
        if t:
            pm["kernels"][k] = {
                "avg_launch_ms": t["avg_launch_ms"], "avg_launch_ms_standalone": t.get("avg_launch_ms_standalone"),
                "probe_avg_launch_ms": t.get("probe_avg_launch_ms"),
                "hbm_bytes_per_launch": t.get("hbm_bytes_per_launch"), "effective_clock_ghz": t.get("effective_clock_ghz"),
                "wave_cycle_split": t.get("wave_cycle_split"),
                "SQ": {n: v for n, v in t["counters_per_launch"].items() if n.startswith("SQ_")}}
    (dst / f"pmc_{cfg['config']}.json").write_text(json.dumps(pm, indent=1) + "\n")
print(json.dumps(summary, indent=1))
