#!/usr/bin/env python3
"""Timeline of single-frame render calls from a rocprofv3 kernel-trace CSV (development aid).

    python3 tools/single_timeline.py run_kernel_trace.csv [--calls 4]

A call starts at its wf_camera launch.  Per call: wall span (first start -> last end), busy time
(union of kernel intervals), and per kernel its start offset, duration and queue/stream id, so
the idle gaps between the passes of a latency-bound frame are visible.
"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("--calls", type=int, default=3)
a = ap.parse_args()

rows = sorted((r for r in csv.DictReader(open(a.csv)) if "rtd::" in r["Kernel_Name"]),
              key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], None
for r in rows:
    if "wf_camera" in r["Kernel_Name"]:
        cur = []
        calls.append(cur)
    if cur is not None:
        cur.append(r)


def short(n):
    n = n.replace("rtd::", "").replace("void ", "").split("(")[0].strip()
    if n.startswith("wf_trace<"):  # <COUNT, WIDE, CAM, STATIC, P1>
        f = [x.strip() == "true" for x in n[len("wf_trace<"):-1].split(",")]
        f += [False] * (5 - len(f))
        return ("trace_cnt" if f[0] else "trace") + ("_cam" if f[2] else "") + ("_p1" if f[4] else "") + ("_s" if f[3] else "")
    return n.replace("wf_shade<true, true>", "shade_fb").replace("wf_shade<true, false>", "shade") \
            .replace("wf_shade<false, true>", "shade_brdf_fb").replace("wf_shade<false, false>", "shade_brdf")


spans = []
for ci, c in enumerate(calls[-a.calls:]):
    t0 = int(c[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in c)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in c)
    busy, s, e = 0, iv[0][0], iv[0][1]
    for x, y in iv[1:]:
        if x > e:
            busy += e - s
            s, e = x, y
        else:
            e = max(e, y)
    busy += e - s
    spans.append((t1 - t0) / 1e3)
    print(f"call {ci}: span {(t1 - t0) / 1e3:8.1f} us  busy {busy / 1e3:8.1f} us  kernels {len(c)}")
    for r in c:
        st, en = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        print(f"   q{q:>3} {short(r['Kernel_Name']):<14} start {st / 1e3:8.1f}  dur {(en - st) / 1e3:7.1f}")
if spans:
    print(f"mean span over {len(spans)} calls: {sum(spans) / len(spans):.1f} us")
