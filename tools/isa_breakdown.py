#!/usr/bin/env python3
"""Static ISA breakdown of one kernel by source region (development aid).

    hipcc ... -gline-tables-only --offload-device-only -S -o rt.s csrc/hip/rt_render.hip
    python3 tools/isa_breakdown.py rt.s <kernel-symbol-regex> [--json out.json]

Every instruction of the kernel is attributed to the source line of its `.loc` (inlined code
keeps its own line), and lines to the function that contains them (a C++ function-header scan of
the csrc/hip headers); per region it reports VALU / SALU / vector-memory / LDS instruction
counts.  Static counts: how often each region runs per ray comes from the COUNT build's visit
counters."""
import argparse
import json
import re
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("asm")
ap.add_argument("kernel")
ap.add_argument("--json")
ap.add_argument("--dump", help="print the instructions of this source function")
a = ap.parse_args()
src_dir = Path(__file__).resolve().parent.parent / "opengl-ray-tracing-framework_amd" / "csrc"

FN = re.compile(r"^(?:template <[^>]*>\s*)?(?:RTD|__global__|GM_FN|inline|static)[^(;]*?\b(\w+)\s*\(")


def regions(path: Path):
    """line -> enclosing function name (a brace-depth scan from each top-level function header)"""
    out, cur, depth = {}, None, 0
    for i, ln in enumerate(path.read_text().splitlines(), 1):
        if ln.startswith("namespace") or ln.startswith("}  // namespace"):
            continue  # namespace braces do not nest functions
        if depth == 0:
            m = FN.match(ln.strip())
            if m:
                cur = m.group(1) if m.group(1) != "__launch_bounds__" else "kernel body"
        depth += ln.count("{") - ln.count("}")
        out[i] = cur if depth > 0 or ln.count("{") else cur
        if depth == 0 and "}" in ln:
            cur = None
    return out


HELPERS = {"dot", "cross", "ld", "mk3", "xyz", "splat", "normalize", "length", "o", "d", "inv", "fabs_", "min_",
           "max_", "ref_is_leaf", "leaf_first", "leaf_count", "pack_ent", "unpack_ent", "sqrt_", "rint_"}
lines = Path(a.asm).read_text().splitlines()
files = {}
for ln in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', ln)
    if m:
        name = m.group(3) or m.group(2)
        files[int(m.group(1))] = Path(name).name
region_maps = {f.name: regions(f) for f in list(src_dir.glob("hip/*.h")) + list(src_dir.glob("hip/*.hip"))
               + list(src_dir.glob("common/*.h"))}
start = next(i for i, ln in enumerate(lines) if re.match(rf"^({a.kernel})\w*:", ln))
kname = lines[start].split(":")[0]
cnt = defaultdict(lambda: defaultdict(int))
loc = ("?", 0)
for ln in lines[start + 1:]:
    if ln.startswith(".Lfunc_end"):
        break
    t = ln.strip()
    m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
    if m:
        # the inline chain in the comment: innermost first; attribute to the innermost frame that
        # is one of our named functions (helpers such as dot / cross / ld roll up to their caller)
        frames = re.findall(r"([\w./-]+\.(?:h|hip)):(\d+):\d+", t.split(";", 1)[1] if ";" in t else "")
        loc = ("?", 0)
        for f, l in frames:
            fn = region_maps.get(Path(f).name, {}).get(int(l))
            if fn and fn not in HELPERS:
                loc = (Path(f).name, int(l))
                break
        continue
    if not t or t.startswith((".", ";")) or t.endswith(":"):
        continue
    op = t.split()[0]
    kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
            "vmem" if op.startswith(("global_", "buffer_", "flat_", "scratch_")) else "lds" if op.startswith("ds_") else "other")
    fn = region_maps.get(loc[0], {}).get(loc[1]) or f"{loc[0]}"
    cnt[fn][kind] += 1
    if a.dump and fn == a.dump:
        print(f"{loc[1]:5d}  {t}")
rows = sorted(cnt.items(), key=lambda kv: -(kv[1]["valu"] + kv[1]["salu"]))
print(f"{kname}: static instructions by source function")
print(f"{'function':28s} {'VALU':>6s} {'SALU':>6s} {'VMEM':>5s} {'LDS':>4s}")
tot = defaultdict(int)
for fn, c in rows:
    print(f"{str(fn):28s} {c['valu']:6d} {c['salu']:6d} {c['vmem']:5d} {c['lds']:4d}")
    for k, v in c.items():
        tot[k] += v
print(f"{'total':28s} {tot['valu']:6d} {tot['salu']:6d} {tot['vmem']:5d} {tot['lds']:4d}")
if a.json:
    Path(a.json).write_text(json.dumps({"kernel": kname, "by_function": {str(k): dict(v) for k, v in rows},
                                        "total": dict(tot)}, indent=1) + "\n")
