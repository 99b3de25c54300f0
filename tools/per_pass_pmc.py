#!/usr/bin/env python3
"""Table of tools/per_pass_pmc.sh: per wf_trace / wf_shade / wf_blend launch of the measured 256-frame
call, its standalone duration, HBM bytes (2 x FETCH_SIZE per the gfx950 note + WRITE_SIZE, kB
counters), the resulting TB/s, VALU issue fraction (1024 SIMDs x 2.4 GHz / 2 cycles) and lane
utilisation."""
import csv
import glob
import sys
from collections import defaultdict

O = sys.argv[1]


def counters(d):
    vals = defaultdict(dict)  # dispatch -> counter -> summed value
    names = {}
    for f in glob.glob(f"{O}/{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = int(r["Dispatch_Id"])
            vals[k][r["Counter_Name"]] = vals[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[k] = r["Kernel_Name"]
    return vals, names


def durations(d):
    out = {}
    for f in glob.glob(f"{O}/{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            out[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return out


def wf_seq(d):
    vals, names = counters(d)
    dur = durations(d)
    seq = [(k, names[k], vals[k], dur.get(k, 0.0)) for k in sorted(vals) if "wf_" in names[k]]
    # the measured call: from the last wf_camera-preceded camera trace (the largest wf_trace<.., true, ..>)
    cam = [i for i, s in enumerate(seq) if "wf_trace" in s[1] and "true, false, false" in s[1].split("<")[1][:40]]
    return seq


f, w, s = wf_seq("f"), wf_seq("w"), wf_seq("s")
n = min(len(f), len(w), len(s))
f, w, s = f[-n:], w[-n:], s[-n:]
print(f"{'kernel':34s} {'ms':>8s} {'fetch GB':>9s} {'write GB':>9s} {'TB/s':>6s} {'VALU issue':>10s} {'lane util':>9s}")
for (kf, name, cf, df), (kw, _, cw, dw), (ks, _, cs, ds) in zip(f, w, s):
    t = ds or df or dw
    if t < 0.05:
        continue
    fe = cf.get("FETCH_SIZE", 0.0) * 2 * 1024 / 1e9
    wr = cw.get("WRITE_SIZE", 0.0) * 1024 / 1e9
    valu = cs.get("SQ_INSTS_VALU", 0.0)
    issue = valu / (1024 * 2.4e9 / 2 * t * 1e-3) if t else 0.0
    act = cs.get("SQ_ACTIVE_INST_VALU", 0.0)
    lane = cs.get("SQ_THREAD_CYCLES_VALU", 0.0) / 64.0 / act if act else 0.0
    short = name.split("(")[0].replace("void ", "").replace("rtd::", "")[:34]
    print(f"{short:34s} {t:8.2f} {fe:9.2f} {wr:9.2f} {(fe + wr) / t:6.2f} {issue:10.3f} {lane:9.3f}")
