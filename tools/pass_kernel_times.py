#!/usr/bin/env python3
"""Durations of each kernel dispatch, in order, from a rocprofv3 --kernel-trace CSV (development aid):
    python3 tools/pass_kernel_times.py gpurun_out/shp/run_kernel_trace.csv [--last N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else len(rows)
t0 = None
for r in rows[-last:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    t0 = s if t0 is None else t0
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    print(f"{name:40s} start {(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f} us  grid {r.get('Grid_Size', '')}")
