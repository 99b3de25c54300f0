#!/usr/bin/env python3
"""Kernel resource table from `make asm` remarks (development aid):
    make -C opengl-ray-tracing-framework_amd asm 2>&1 | python3 tools/kres.py [regex]"""
import re
import sys

pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
cur, rows = None, {}
for ln in sys.stdin:
    m = re.search(r"remark:\s+Function Name: (\S+)", ln)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\S+) \[", ln)
    if m and cur:
        rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    if pat and not pat.search(k):
        continue
    print(f"{k[:64]:64s} vgpr {v.get('VGPRs','?'):>3} sgpr {v.get('TotalSGPRs','?'):>3} scratch {v.get('ScratchSize [bytes/lane]','?'):>3} "
          f"occ {v.get('Occupancy [waves/SIMD]','?')} vspill {v.get('VGPRs Spill','?')} sspill {v.get('SGPRs Spill','?')}")
