#!/usr/bin/env python3
"""Per-pass kernel durations of the wavefront path from a rocprofv3 kernel-trace CSV."""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "wf_" in r["Kernel_Name"]]
groups, cur = [], None
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "wf_camera" in n or ("wf_gen" in n and (cur is None or cur["blend"] or cur["trace"])):
        cur = {"gen": d, "trace": [], "shade": [], "blend": 0.0}  # gen: wf_camera (+ wf_gen)
        groups.append(cur)
    elif "wf_gen" in n:
        cur["gen"] += d
    elif cur is not None:
        if "wf_trace" in n:
            cur["trace"].append(d)
        elif "wf_shade" in n:
            cur["shade"].append(d)
        elif "wf_blend" in n:
            cur["blend"] = d
for i, g in enumerate(groups):
    tot = g["gen"] + sum(g["trace"]) + sum(g["shade"]) + g["blend"]
    print(f"group {i}: total {tot:8.1f} us  gen {g['gen']:.0f}  blend {g['blend']:.0f}")
    print("   trace: " + " ".join(f"{x:6.0f}" for x in g["trace"]) + f"   sum {sum(g['trace']):.0f}")
    print("   shade: " + " ".join(f"{x:6.0f}" for x in g["shade"]) + f"   sum {sum(g['shade']):.0f}")
