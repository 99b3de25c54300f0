#!/usr/bin/env python3
"""Aggregate rocprofv3 counter CSVs per kernel name (sum over dispatches)."""
import csv
import glob
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
for f in glob.glob(sys.argv[1] + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:32]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    if "rocclr" in k:
        continue
    print(k)
    for n in sorted(c):
        print(f"   {n:28s} {c[n]:.4g}")
    if c.get("SQ_ACTIVE_INST_VALU"):
        print(f"   -> VALU lane util {c['SQ_THREAD_CYCLES_VALU'] / (c['SQ_ACTIVE_INST_VALU'] * 64):.3f}")
    if c.get("SQ_WAVE_CYCLES"):
        w = c["SQ_WAVE_CYCLES"]
        print(f"   -> wait_any {c['SQ_WAIT_ANY']/w:.2f} wait_inst {c['SQ_WAIT_INST_ANY']/w:.2f} active {c['SQ_ACTIVE_INST_ANY']/w:.2f}")
    if c.get("TCC_HIT_sum"):
        print(f"   -> L2 hit {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}")
