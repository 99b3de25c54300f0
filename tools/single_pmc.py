#!/usr/bin/env python3
"""Per-kernel SQ summary of tools/single_pmc.sh's two PMC passes (development aid).

Per kernel (all dispatches of the run, standalone under counter collection): mean duration,
waves, instructions per wave by kind, and the wave-cycle split (SQ_WAVE_CYCLES, SQ_WAIT_ANY,
SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY count quad-cycles per the MI355X guide)."""
import csv
import statistics
import sys
from collections import defaultdict
from pathlib import Path

src = Path(sys.argv[1])


def short(n):
    n = n.replace("rtd::", "").split("(")[0]
    return n.replace("void ", "").strip()


vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))  # kernel -> dispatch -> counter
durs = defaultdict(dict)
for p in ("sq", "sq2"):
    f = src / p / "run_counter_collection.csv"
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        vals[k][(p, r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    t = src / p / "run_kernel_trace.csv"
    if t.exists():
        for r in csv.DictReader(open(t)):
            durs[short(r["Kernel_Name"])][(p, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for k in sorted(vals):
    c = defaultdict(list)
    for d in vals[k].values():
        for n, v in d.items():
            c[n].append(v)
    m = {n: statistics.mean(v) for n, v in c.items()}
    waves = m.get("SQ_WAVES", 0) or 1
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    us = statistics.mean(durs[k].values()) if durs.get(k) else 0
    print(f"{k}: {us:.1f} us standalone, {m.get('SQ_WAVES', 0):.0f} waves; per wave VALU {m.get('SQ_INSTS_VALU', 0) / waves:.0f} "
          f"SALU {m.get('SQ_INSTS_SALU', 0) / waves:.0f} LDS {m.get('SQ_INSTS_LDS', 0) / waves:.0f} "
          f"VMEM_RD {m.get('SQ_INSTS_VMEM_RD', 0) / waves:.0f} SMEM {m.get('SQ_INSTS_SMEM', 0) / waves:.0f} "
          f"BRANCH {m.get('SQ_INSTS_BRANCH', 0) / waves:.0f}; wave cycles: issuing {m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} "
          f"waiting {m.get('SQ_WAIT_ANY', 0) / wc:.3f} issue-stalled {m.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}; "
          f"VALU active {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f} SALU {m.get('SQ_ACTIVE_INST_SCA', 0) / wc:.3f} "
          f"LDS {m.get('SQ_ACTIVE_INST_LDS', 0) / wc:.3f}; lane util "
          f"{m.get('SQ_THREAD_CYCLES_VALU', 0) / (64 * (m.get('SQ_ACTIVE_INST_VALU', 0) or 1)):.3f}; "
          f"mean wave life {4 * wc / waves / 2400:.1f} us at 2.4 GHz")
