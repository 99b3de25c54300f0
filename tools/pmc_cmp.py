#!/usr/bin/env python3
"""Summarise tools/pmc_cmp.sh: per variant and kernel, the summed durations and counters, VALU
issue fraction (4 cycles per wave64 VALU instruction on a 16-lane SIMD, 1024 SIMDs), lane
utilisation, L2 hit rate."""
import csv
import glob
import sys
from collections import defaultdict


def kname(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].replace("rtd::", "")


root, variants = sys.argv[1], sys.argv[2:]
for v in variants:
    dur = defaultdict(float)
    for f in glob.glob(f"{root}/{v}/t/**/run_kernel_trace.csv", recursive=True) + glob.glob(f"{root}/{v}/t/run_kernel_trace.csv"):
        for r in csv.DictReader(open(f)):
            dur[kname(r)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    cnt = defaultdict(lambda: defaultdict(float))
    for p in ("a", "b", "c"):
        for f in set(glob.glob(f"{root}/{v}/{p}/**/run_counter_collection.csv", recursive=True) +
                     glob.glob(f"{root}/{v}/{p}/run_counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                cnt[kname(r)][r["Counter_Name"]] += float(r["Counter_Value"])
    rays = 0
    for ln in open(f"{root}/{v}.a.log", errors="replace"):
        if ln.startswith("rays_total "):
            rays = int(ln.split()[1])
    print(f"== {v}" + (f"  ({rays} rays, every render of the run)" if rays else ""))
    for k in sorted(dur, key=lambda k: -dur[k]):
        if not k.startswith("wf_") and "rt_" not in k:
            continue
        c = cnt.get(k, {})
        line = f"  {k:12s} {dur[k]:9.2f} ms"
        if c.get("SQ_INSTS_VALU"):
            cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
            line += f"  valu {c['SQ_INSTS_VALU']:.3e}"
            if cyc:
                line += f"  issue {c['SQ_INSTS_VALU'] * 4 / (1024 * cyc):.3f}  clk {cyc / (dur[k] * 1e6):.2f}GHz"
            if c.get("SQ_ACTIVE_INST_VALU"):
                line += f"  lanes {c['SQ_THREAD_CYCLES_VALU'] / (64 * c['SQ_ACTIVE_INST_VALU']):.3f}"
            if c.get("SQ_WAVE_CYCLES"):
                line += f"  wait {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.2f}"
            line += f"  vmem {c.get('SQ_INSTS_VMEM_RD', 0):.3e}  salu {c.get('SQ_INSTS_SALU', 0):.3e}"
            if rays and k == "wf_trace":
                line += (f"  per ray: valu {c['SQ_INSTS_VALU'] / rays:.1f} salu {c.get('SQ_INSTS_SALU', 0) / rays:.1f}"
                         f"  salu/valu {c.get('SQ_INSTS_SALU', 0) / c['SQ_INSTS_VALU']:.2f}")
        if c.get("WRITE_SIZE"):  # KB (MI355X_MICROARCH.md)
            line += f"  write {c['WRITE_SIZE'] * 1024 / 1e9:.2f} GB"
            if rays and k == "wf_trace":
                line += f" ({c['WRITE_SIZE'] * 1024 / rays:.1f} B written per ray)"
        if c.get("TCC_HIT_sum"):
            line += f"  L2hit {c['TCC_HIT_sum'] / (c['TCC_HIT_sum'] + c['TCC_MISS_sum']):.3f}"
        print(line)
