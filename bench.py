#!/usr/bin/env python3
"""bench.py — Mrays/sec + ms/frame of the MI355X path tracer (BASELINE.json metric).

Workload (default): config C3 = floor + loong_100000 (copper), 1920x1080, maxBounce 8,
HDR-environment MIS, camera/material/RNG exactly as the reference (rtamd/configs.py).
One *step* = ``--frames-per-step`` (default 1024 = the C3 config's spp)
progressive frames (1 spp each) of the whole frame, rendered by one rt_render call per rank
over that rank's pixel tiles with as many frames in flight as HBM holds (rt_set_max_paths:
184 B per pixel-frame; one GPU runs the step as two launches of 512 frames = 206 GB of path
state each, 8 tile-sharded GPUs run it as one launch of 1024 frames = 51 GB per rank),
followed by the frame-end gather of every rank's fp32 accumulation tiles to rank 0 (RCCL over
xGMI via torch.distributed, backend "nccl") and the un-permute into the full frame on rank 0.

    python bench.py [--gpus 1] [--steps 10] [--warmup 2]
    python bench.py --gpus N ...          (spawns N rank processes itself, one per GPU)
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
    python bench.py --dry-run --gpus 2    (CPU: launcher, frame plan and gloo gather only)

Rank 0 prints ONE JSON line.  value = rays traced by all ranks / max-over-ranks wall time
of the timed steps (barrier + synchronize on both sides).  Rays are counted on the device
(camera + NEE shadow + continuation = every hitBVH call of the reference, RT:1386/1480/1528).
randOrigin_k for any number of frames comes from the in-tree restatement of glibc rand()
(main.cpp:190, rtamd/configs.py rand_origins).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "opengl-ray-tracing-framework_amd"))

import numpy as np  # noqa: E402

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"]
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)
L2_PEAK_GBS = 34500.0     # aggregate L2 bandwidth, measured (MI355X_MICROARCH.md §L2)
N_SIMD = 256 * 4          # CUs x SIMDs
VALU_CYC = 2              # cycles per wave64 VALU instruction (MI355X_MICROARCH.md: 32 lanes/cycle x 2)
SPEC_CLOCK_GHZ = 2.4      # max engine clock (MI355X_MICROARCH.md chip-level parameters)
# algorithmic bytes per traversal from the reference's visit counts
#   64 B per internal pop (16 B node ints + two 24-B child AABBs), 16 B per leaf pop,
#   36 B per triangle test (positions), 132 B per closer-hit update (normals + material),
#   12 B per HDR texel fetch, 12 B per cache texel fetch, + 24 B per pixel-frame (accum r/w)
B_INT, B_LEAF, B_TRI, B_UPD, B_ENV, B_CACHE, B_PIXEL = 64, 16, 36, 132, 12, 12, 24
# wf_trace's own HBM stream per ray (the ~25 MB scene stays in L2 / Infinity Cache): a
# secondary ray reads its 4-B queue entry and its 24-B origin/direction (WFState ra/rb or sa/sb:
# {o.xyz, d.x} float4 + {d.y, d.z} float2) and writes its 4-B result (the closest triangle; the
# shade recomputes t); a camera ray is rebuilt from the per-pixel camera table (16 B per pixel,
# shared by the pixel's frames) and writes its 4-B result; pass 1's rays (rt_stats.p1_rays) are
# 16-B records {d, scattering distance} whose origin is the pixel's camera hit point (WFState org,
# 16 B per pixel, shared by the pixel's frames) (tests/test_bench_cpu.py pins these to the WFState
# layout)
B_RAY_SECONDARY, B_RAY_PASS1, B_RAY_CAMERA = 4 + 24 + 4, 4 + 16 + 4, 4
# wf_trace's own traversal bytes per visit (served from L2 / MALL): a 128-B 4-wide node, a
# 48-B triangle record
B_QNODE, B_TRI_REC = 128, 48


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--frames-per-step", type=int, default=1024)
    ap.add_argument("--tile", type=int, default=0,
                    help="pixel tile edge of the rank shares (0: 32 at N = 1, 16 at N > 1: the cost-balanced "
                         "map of 16-px tiles evens the 8 ranks out better, max/mean 1.006-1.009 vs 1.014-1.015, "
                         "DESIGN §5 round 5; N = 1 unchanged)")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bounded CPU-baseline sample: oracle frames until this wall time (0 disables)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--single-frames", type=int, default=64,
                    help="frames rendered one per rt_render call after the timed region (ms_per_frame_single)")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="render calls in flight together (rt_set_pipeline; 1: off): the one-frame calls of "
                         "ms_per_frame_single (and the steps with --pipeline-steps)")
    ap.add_argument("--pipeline-steps", action="store_true",
                    help="steps in flight together too (two steps' path state: at N = 1 --frames-per-step <= 256 at 1080p)")
    ap.add_argument("--no-gather", action="store_true", help="skip the frame-end gather (diagnostics only)")
    ap.add_argument("--no-balance", action="store_true",
                    help="N > 1: keep the interleaved t %% N tile map instead of the cost-balanced one")
    ap.add_argument("--rehearse", action="store_true",
                    help="N > 1 on ONE GPU: every rank on device 0, collectives over gloo on host copies "
                         "(tests the multi-rank render, balance, gather and assembly without RCCL)")
    ap.add_argument("--frame-sha", action="store_true",
                    help="rank 0 adds the sha256 of the assembled fp32 frame after the timed steps")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: launcher, frame plan, tiling and the gloo gather only (CPU tests)")
    ap.add_argument("--fail-rank", type=int, default=-1,
                    help="(with --dry-run) this rank exits with status 3 before the rendezvous (launcher test)")
    a = ap.parse_args(argv)
    if a.tile <= 0:
        a.tile = 16 if a.gpus > 1 else 32
    return a


# ------------------------------------------------------------------------------ launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` without a torch.distributed launcher: start N rank processes (one per
    GPU) with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, wait for all, and forward rank 0's
    JSON line.  This parent never touches the GPU (no torch import), so nothing is initialised
    in it before the children start."""
    port = _free_port()
    procs = []
    out0 = tempfile.TemporaryFile(mode="w+")  # rank 0's stdout (a file: no pipe to drain while polling)
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n), "LOCAL_WORLD_SIZE": str(n),
                    "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL, text=True))
    # fail fast: a rank that dies leaves the others blocked in a collective (or the rendezvous)
    # until its timeout, so the first non-zero exit stops the ranks still running
    rcs = [None] * n
    first_fail = None
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] and first_fail is None:
                    first_fail = rcs[i]
        if first_fail is not None:
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.2)
    out0.seek(0)
    line = next((ln for ln in reversed(out0.read().splitlines()) if ln.startswith("{")), None)
    out0.close()
    if any(rcs) or line is None:
        print(f"bench.py: rank exit codes {rcs}" + ("" if line else "; rank 0 printed no JSON line"),
              file=sys.stderr)
        return first_fail or next((rc for rc in rcs if rc), 1)
    print(line, flush=True)
    return 0


# ------------------------------------------------------------------------------ CPU baseline
def host_cpus() -> dict:
    """The host's cores as this process sees them: the machine's logical CPUs (nproc), the ones
    this process may run on (affinity), a cgroup CPU quota if one is set, OMP_NUM_THREADS and the
    CPU model."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = info["nproc"]
    try:
        q, per = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    omp = os.environ.get("OMP_NUM_THREADS", "")
    info["omp_num_threads"] = int(omp) if omp.isdigit() else None
    try:
        for ln in Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                info["cpu_model"] = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def cpu_baseline(sd, env, W, H, fp, seconds: float, threads: int):
    """The oracle (CPU restatement of the shader, OpenMP) on whole frames 1..k of the same
    workload until `seconds` of wall time; returns the JSON object and the §8(d) counters.
    Threads: --cpu-threads, else every CPU this process may run on, bounded by the CPU share the
    host grants it (the cgroup quota, or OMP_NUM_THREADS where the pool sets the share that way:
    16 per GPU on the MI355X pool); the object records all of them."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle as orc  # cpu_baseline leg only: the checker, timed as the reference-algorithm baseline
    from rtamd import configs as cf

    host = host_cpus()
    if threads <= 0:
        threads = host["affinity"]
        if host["cgroup_cpu_quota"]:
            threads = min(threads, max(1, int(host["cgroup_cpu_quota"])))
        if host["omp_num_threads"]:
            threads = min(threads, host["omp_num_threads"])
    scene = orc.OracleScene(sd.tri_enc, sd.node_enc, env[0], env[1])
    ro = cf.rand_origins(32)
    acc = None
    tot = None
    t0 = time.perf_counter()
    k = 0
    while k < 32:
        acc, cnt = orc.render(scene, [cf.oracle_frame_params(fp, k + 1, ro[k])], W, H, accum=acc, threads=threads)
        tot = cnt if tot is None else {key: tot[key] + cnt[key] for key in tot}
        k += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    value = tot["rays"] / dt / 1e6
    obj = {"value": round(value, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
           "sample": f"oracle/rt_oracle.cpp (CPU restatement of the GLSL path, no culling) on {k} full "
                     f"{W}x{H} frame(s) of the same workload, {tot['rays']} rays in {dt:.1f} s on {threads} "
                     "OpenMP threads; llvmpipe GL baseline unavailable (no GL/EGL context, SURVEY §8(c))",
           "ms_per_frame": round(dt * 1e3 / k, 1),
           "per_core": round(value / threads, 3),
           "host": host}
    return obj, tot


# ------------------------------------------------------------------------------ roofline
def load_profile(config: str, W: int, H: int, F: int, slots: int):
    """profiles/pmc_<config>.json (tools/profile_gpu.sh + tools/summarize_profile.py): rocprofv3
    kernel-trace durations and PMC counters of the bench workload's wf_trace and wf_shade
    launches; used only when its workload key matches this run."""
    p = ROOT / "profiles" / f"pmc_{config}.json"
    if not p.exists():
        return None
    d = json.loads(p.read_text())
    if (d.get("width") == W and d.get("height") == H and d.get("frames_per_step") == F
            and d.get("path_slots_per_rank") == slots and "kernels" in d):
        d["_file"] = str(p.relative_to(ROOT))
        return d
    return None


# wf_shade's algorithmic HBM bytes per path step (one path shaded in one bounce pass; rt_wavefront.h
# shade_path, path-state layout DESIGN.md §3), for a path that continues with a shadow ray and a
# continuation.  Passes >= 2: it reads its active-list entry (4 B), s5 (8), s0 + s2 (32), its two
# 4-B results (8) and its 24-B continuation ray = 76 B, and writes s0 + s2 + s5 (40), the next
# continuation and shadow rays (2 x 24), two queue entries and an active entry (12) = 100 B.
# Pass 0 (implicit camera paths): reads only the camera ray's 4-B result and writes the 16-B ray
# records {d, s} of pass 1 (2 x 16) = 4 + 84 B.  Pass 1: reads the 16-B continuation record
# instead of 24 B = 68 + 100 B.  The s1 / s3 / s4 rows (Lo, NEE, medium terms) are not counted
# (PF_ZLO paths skip them), nor the final colour of finishing paths.  Path steps per pass come
# from the device (rt_stats.pass0_steps / pass1_steps / path_steps; the finisher's steps,
# rt_stats.finish_steps, run in wf_finish and are not wf_shade's).
B_SHADE_STEP = 76 + 100
B_SHADE_P0 = 4 + 40 + 2 * 16 + 12
B_SHADE_P1 = 68 + 100
VALU_PEAK_G = N_SIMD * SPEC_CLOCK_GHZ / VALU_CYC  # G wave64-VALU-instructions/s (2 cycles each per SIMD)


def shade_bytes(st) -> float:
    """wf_shade's algorithmic bytes over the counted path steps (see B_SHADE_*)."""
    p0, p1 = st.get("pass0_steps", 0), st.get("pass1_steps", 0)
    rest = max(0, st["path_steps"] - p0 - p1)
    return B_SHADE_P0 * p0 + B_SHADE_P1 * p1 + B_SHADE_STEP * rest


def trace_bytes(st) -> float:
    """wf_trace's algorithmic HBM bytes over all its launches (B_RAY_*): camera rays (one per
    sample), pass-1 rays (rt_stats.p1_rays) and the other secondary rays."""
    cam, p1 = st["samples"], st.get("p1_rays", 0)
    return B_RAY_SECONDARY * (st["rays"] - cam - p1) + B_RAY_PASS1 * p1 + B_RAY_CAMERA * cam


def roofline(st, vis, cnt, prof, probe, steps):
    """wf_trace, the dominant kernel, priced against the roofline of what bounds it.

    Time per launch = the STANDALONE launch (`probe`: the same per-launch workload rendered as one
    frame group, RT_FLAG_SERIAL, so no other kernel shares the CUs; HIP events on the launch
    stream).  The timed region runs two frame groups whose launches overlap, so co-running per-launch
    times would add up to more than the step (bench line `kernel`); this regime never does.
    Utilisations at that time: HBM (algorithmic bytes: the path-state stream the kernel must move,
    B_RAY_*; the ~25 MB scene stays in L2 / MALL), VALU issue (PMC VALU instructions per launch vs
    1024 SIMDs x 2.4 GHz / 2 cycles) and L2 (its own traversal bytes).  `bound` is the largest of
    them and achieved / peak / unit / frac are that roofline's; the others are given beside it
    (`hbm`, `valu`, `l2`).  `traffic` = rocprofv3 PMC HBM bytes per launch.  `kernels.wf_shade`:
    the memory-bound shade against the HBM peak.  `reference_equivalent`: SURVEY §8(d)'s bytes of
    the reference's exhaustive traversal, labelled as such and never used as frac."""
    launches = max(1, st["trace_launches"])
    rays_l = st["rays"] / launches
    src = probe if (probe and probe.get("trace_launches")) else None
    if src:
        t_ms = src["trace_ms"] / src["trace_launches"]
        alg = trace_bytes(src) / src["trace_launches"]
        regime = (f"standalone: the probe render of {src.get('frames')} frames as one frame group (RT_FLAG_SERIAL), "
                  f"{src['trace_launches']} launches, HIP events on the launch stream")
    else:  # no probe: the co-running launches (labelled)
        t_ms = st["trace_ms"] / launches
        alg = trace_bytes(st) / launches
        regime = "co-running (two frame groups overlap; per-launch times add up to more than the step)"
    sec = t_ms * 1e-3
    hbm = {"achieved": round(alg / sec / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(alg / sec / 1e9 / HBM_PEAK_GBS, 4), "algorithmic_bytes_per_launch": round(alg),
           "algorithmic_bytes_per_ray": {"secondary": B_RAY_SECONDARY, "pass1": B_RAY_PASS1, "camera": B_RAY_CAMERA}}
    out = {"bound": "hbm", "achieved": hbm["achieved"], "peak": hbm["peak"], "unit": hbm["unit"], "frac": hbm["frac"],
           "traffic": None, "kernel": "wf_trace", "avg_launch_ms": round(t_ms, 4), "avg_launch_ms_regime": regime,
           "launches_per_step": round(launches / max(1, steps), 2),
           "rays_per_launch": round(src["rays"] / src["trace_launches"]) if src else round(rays_l),
           "hbm": hbm}
    util = {"hbm": hbm["frac"]}
    pt = (prof or {}).get("kernels", {}).get("wf_trace")
    if pt:
        out["traffic"] = pt.get("hbm_bytes_per_launch")
        out["profile"] = prof["_file"]
        out["profile_avg_launch_ms_standalone"] = pt.get("probe_avg_launch_ms") or pt.get("avg_launch_ms_standalone")
        out["profile_avg_launch_ms_corunning"] = pt.get("avg_launch_ms")
        sq = pt.get("SQ", {})
        if sq.get("SQ_INSTS_VALU"):
            ach = sq["SQ_INSTS_VALU"] / sec / 1e9
            v = {"achieved": round(ach, 1), "peak": round(VALU_PEAK_G, 1), "unit": "G VALU wave-instr/s",
                 "frac": round(ach / VALU_PEAK_G, 4), "insts_per_launch": round(sq["SQ_INSTS_VALU"]),
                 "insts_per_ray": round(sq["SQ_INSTS_VALU"] / rays_l, 1), "cycles_per_inst": VALU_CYC,
                 "spec_clock_ghz": SPEC_CLOCK_GHZ}
            if sq.get("SQ_INSTS_SALU"):
                v["salu_per_ray"] = round(sq["SQ_INSTS_SALU"] / rays_l, 1)
                v["salu_per_valu"] = round(sq["SQ_INSTS_SALU"] / sq["SQ_INSTS_VALU"], 3)
            if pt.get("effective_clock_ghz"):
                v["effective_clock_ghz"] = pt["effective_clock_ghz"]
            if sq.get("SQ_ACTIVE_INST_VALU") and sq.get("SQ_THREAD_CYCLES_VALU"):
                v["lane_util"] = round(sq["SQ_THREAD_CYCLES_VALU"] / (64 * sq["SQ_ACTIVE_INST_VALU"]), 4)
            if pt.get("wave_cycle_split"):
                v["wave_cycle_split"] = pt["wave_cycle_split"]
            out["valu"] = v
            util["valu_issue"] = v["frac"]
    if vis and vis.get("rays"):
        own = (B_QNODE * vis["internal_pops"] + B_TRI_REC * vis["tri_tests"]) / vis["rays"]
        rl = src["rays"] / src["trace_launches"] if src else rays_l
        out["l2"] = {"own_traversal_bytes_per_ray": round(own, 1), "achieved": round(own * rl / sec / 1e9, 1),
                     "peak": L2_PEAK_GBS, "unit": "GB/s", "frac": round(own * rl / sec / 1e9 / L2_PEAK_GBS, 4)}
        util["l2"] = out["l2"]["frac"]
    lim = max(util, key=util.get)
    out["utilisation"] = util
    out["limiter"] = lim
    if lim == "valu_issue":
        v = out["valu"]
        out.update(bound="valu_issue", achieved=v["achieved"], peak=v["peak"], unit=v["unit"], frac=v["frac"])
    elif lim == "l2":
        l2 = out["l2"]
        out.update(bound="l2", achieved=l2["achieved"], peak=l2["peak"], unit=l2["unit"], frac=l2["frac"])
    if cnt:
        per_ray = (B_INT * cnt["internal_pops"] + B_LEAF * cnt["leaf_pops"] + B_TRI * cnt["tri_tests"] +
                   B_UPD * cnt["closer_updates"]) / cnt["rays"]
        out["reference_equivalent"] = {
            "bytes_per_ray": round(per_ray, 1), "gbs": round(per_ray * rays_l / sec / 1e9, 1),
            "note": "SURVEY §8(d) bytes of the reference's own exhaustive traversal (oracle visit counts) per "
                    "ray traced here; the device traversal visits fewer nodes, so this is not a bandwidth"}
    ps = (prof or {}).get("kernels", {}).get("wf_shade")
    if ps and ps.get("avg_launch_ms_standalone") and st.get("path_steps"):
        alg_s = shade_bytes(st) / launches  # one wf_shade per wf_trace launch
        t_s = ps["avg_launch_ms_standalone"] * 1e-3
        out["kernels"] = {"wf_shade": {
            "bound": "hbm", "achieved": round(alg_s / t_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(alg_s / t_s / 1e9 / HBM_PEAK_GBS, 4), "traffic": ps.get("hbm_bytes_per_launch"),
            "traffic_frac": (round(ps["hbm_bytes_per_launch"] / t_s / 1e9 / HBM_PEAK_GBS, 4)
                             if ps.get("hbm_bytes_per_launch") else None),
            "avg_launch_ms_standalone": ps["avg_launch_ms_standalone"],
            "launches_per_step": round(launches / max(1, steps), 2),
            "algorithmic_bytes_per_launch": round(alg_s),
            "algorithmic_bytes_per_path_step": {"pass0": B_SHADE_P0, "pass1": B_SHADE_P1, "later": B_SHADE_STEP},
            "path_steps_per_launch": round(st["path_steps"] / launches),
            "note": "algorithmic bytes of a continuing path's step (s1/s3/s4 rows and final colours not counted); "
                    "time = the PMC passes' standalone launches (dispatches serialised), the visit-count frame's "
                    "launches excluded",
            "profile": prof["_file"]}}
    return out


# ------------------------------------------------------------------------------ dry run
def dry_run(args, rank: int, world: int) -> int:
    """CPU rehearsal of the multi-rank bench: frame plan (randOrigin for every frame), each
    rank's tile share, and the frame-end gather over gloo with max-over-ranks timing."""
    import torch
    import torch.distributed as dist

    from rtamd import configs as cf
    from rtamd import tiling

    cfg = cf.CONFIGS[args.config]
    W, H = args.width or cfg.width, args.height or cfg.height
    F, steps, warm = args.frames_per_step, args.steps, args.warmup
    total_frames = (warm + steps) * F + 1 + args.single_frames
    if rank == args.fail_rank:
        print(f"bench.py: rank {rank} fails on purpose (--fail-rank)", file=sys.stderr)
        return 3
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    ro = cf.rand_origins(total_frames)
    owner = None
    if world > 1 and not args.no_balance:
        # the GPU run measures per-tile costs with rt_tile_costs; here a synthetic stand-in
        # through the same exchange (all_reduce of each rank's share) and the same balance()
        n_t = len(tiling.modulo_owners(W, H, args.tile, args.tile, world))
        full = torch.zeros(n_t, dtype=torch.int64)
        for t in tiling.local_tiles(W, H, args.tile, args.tile, rank, world):
            full[t] = (t * 7919) % 1000 + 1
        dist.all_reduce(full)
        owner = tiling.balance(full.numpy(), world)
    mine = tiling.local_tiles(W, H, args.tile, args.tile, rank, world, owner)
    mlt = tiling.max_local_tiles(W, H, args.tile, args.tile, world, owner)
    px = sum(tiling.tile_rect(t, W, H, args.tile, args.tile)[2] * tiling.tile_rect(t, W, H, args.tile, args.tile)[3]
             for t in mine)
    t0 = time.perf_counter()
    local = torch.full((mlt, 4), float(rank))
    if world > 1:
        parts = [torch.empty_like(local) for _ in range(world)] if rank == 0 else None
        dist.gather(local, gather_list=parts, dst=0)
        pxs = torch.tensor([float(px)])
        dist.all_reduce(pxs)
        elapsed = torch.tensor([time.perf_counter() - t0])
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        total_px = int(pxs[0])
        ok = rank != 0 or all(int(p[0, 0]) == r for r, p in enumerate(parts))
    else:
        total_px, ok, elapsed = px, True, torch.tensor([time.perf_counter() - t0])
    rank_ms = [round(float(elapsed[0]) * 1e3, 3)] * world
    if world > 1:  # each rank's own time (the same all-gather the GPU run's line uses)
        mine = torch.tensor([(time.perf_counter() - t0) * 1e3], dtype=torch.float64)
        everyone = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(everyone, mine)
        rank_ms = [round(float(t[0]), 3) for t in everyone]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mrays/s", "n_gpus": world, "steps": steps,
                          "warmup": warm, "dry_run": True, "frames_planned": total_frames,
                          "rand_origin_last": float(ro[-1]), "pixels_covered": total_px,
                          "frame_pixels": W * H, "gather_ok": bool(ok),
                          "tile_assignment": "modulo" if owner is None else "cost-balanced",
                          "gather_ms": round(float(elapsed[0]) * 1e3, 3),
                          "collective": {"backend": dist.get_backend() if world > 1 else None, "world": world,
                                         "gather_ms": round(float(elapsed[0]) * 1e3, 3), "rank_ms": rank_ms}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0 if (total_px == W * H and ok) else 1


# ------------------------------------------------------------------------------ bench
def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(args, rank, world)
    import torch
    dist = None
    dev = 0 if args.rehearse else local_rank
    torch.cuda.set_device(dev)
    cdev = "cpu" if args.rehearse else "cuda"  # where the collectives' tensors live
    if world > 1:
        import torch.distributed as dist
        if args.rehearse:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))

    from rtamd import configs as cf
    from rtamd.renderer import RT_FLAG_COUNT_VISITS, Renderer

    cfg = cf.CONFIGS[args.config]
    W, H = args.width or cfg.width, args.height or cfg.height
    F, steps, warm = args.frames_per_step, args.steps, args.warmup
    n_single = max(0, args.single_frames)
    total_frames = (warm + steps) * F + 1 + n_single
    sd = cf.config_scene(args.config)
    env = cf.load_env()
    fp = cf.frame_params(W, H)
    ro = cf.rand_origins(total_frames)

    # One stream for everything: the renderer's kernels and copies and torch's RCCL collectives
    # (ProcessGroupNCCL orders its internal stream after the *current* stream), so the gather reads
    # finished tiles and the assemble reads the gathered ones.
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    r = Renderer(dev)
    r.set_stream(stream.cuda_stream)
    r.set_scene_soa(sd.soa, sd.nodes)
    r.set_env(*env)
    r.resize(W, H, tile=args.tile, rank=rank, world=world)
    balanced = world > 1 and not args.no_balance
    if balanced:
        # tiles assigned by a cost estimate from one probe frame.  Every rank measures
        # its interleaved share (rt_tile_costs: node + triangle steps per tile), the shares are
        # summed into the full cost vector, and every rank derives the same LPT owner map
        from rtamd import tiling
        n_t = len(tiling.modulo_owners(W, H, args.tile, args.tile, world))
        full = torch.zeros(n_t, dtype=torch.int64, device=cdev)
        mine = torch.tensor(tiling.local_tiles(W, H, args.tile, args.tile, rank, world), dtype=torch.int64,
                            device=cdev)
        full[mine] = torch.from_numpy(r.tile_costs(fp, ro[-1:]).astype(np.int64)).to(cdev)
        dist.all_reduce(full)
        r.set_tile_owners(tiling.balance(full.cpu().numpy(), world))
    # --pipeline-steps: consecutive steps in flight together (rt_set_pipeline: each step's launch on
    # its own stream and path-state set, only its blend ordered after the previous step and the
    # gather).  Off by default: in steady state (step k+2 waits for step k) a rank's share at N = 8
    # measured the same (tools/rank_sim.py --pipeline 2, 3 steps: 81.7 vs 81.6 ms), and one GPU runs
    # a step as two launches whose state fills the HBM once.
    pipelined = args.pipeline > 1 and args.pipeline_steps
    if pipelined:
        r.set_pipeline(args.pipeline)
    ad = r.accum_device()
    # path-state budget: a whole step's frames in flight at once (184 B per pixel-frame: 51 GB
    # per rank for 1024 frames of 1080p at N = 8); the library halves the frames per launch
    # until the state fits (512 = 206 GB of HBM3E on one GPU)
    path_slots = F * ad["local_tiles"] * args.tile * args.tile
    r.set_max_paths(path_slots)
    nfloat = ad["bytes"] // 4
    local = torch.empty(nfloat, dtype=torch.float32, device="cuda")
    gathered = torch.empty(world * nfloat, dtype=torch.float32, device="cuda") if rank == 0 else None
    frame = torch.empty(H * W * 3, dtype=torch.float32, device="cuda") if rank == 0 else None

    gather_ev = []  # (start, end) CUDA events around each step's frame-end gather on this rank's stream

    def step(k: int) -> None:
        r.render_async(fp, ro[k * F:(k + 1) * F])
        if args.no_gather:
            return
        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        gather_ev.append(ev)
        ev[0].record()  # (runs once this step's render has finished: same stream)
        if world == 1:
            r.assemble_frame(ad["ptr"], 1, frame.data_ptr())
            ev[1].record()
            return
        r.copy_accum_device(local.data_ptr(), ad["bytes"])
        if args.rehearse:  # gloo: host copies
            parts = [torch.empty(nfloat, dtype=torch.float32) for _ in range(world)] if rank == 0 else None
            dist.gather(local.cpu(), gather_list=parts, dst=0)
            if rank == 0:
                gathered.copy_(torch.cat(parts))
        else:
            parts = list(gathered.view(world, nfloat).unbind(0)) if rank == 0 else None
            dist.gather(local, gather_list=parts, dst=0)
        if rank == 0:
            r.assemble_frame(gathered.data_ptr(), world, frame.data_ptr())
        ev[1].record()  # (the current stream waited for the collective's stream: async_op=False)

    t_w = time.perf_counter()
    for k in range(warm):
        step(k)
    torch.cuda.synchronize()
    if rank == 0:
        print(f"bench: warmup {warm} x {F} frames in {time.perf_counter() - t_w:.1f} s", file=sys.stderr, flush=True)
    r.reset_stats()
    gather_ev.clear()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(warm, warm + steps):
        step(k)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = r.stats()
    gather_ms = (sum(a.elapsed_time(b) for a, b in gather_ev) / len(gather_ev)) if gather_ev else 0.0
    rank_elapsed = elapsed

    # whole-job aggregates
    vals = torch.tensor([elapsed, float(st["rays"]), float(st["samples"])], dtype=torch.float64, device=cdev)
    per_rank = torch.tensor([rank_elapsed * 1e3 / max(1, steps), gather_ms], dtype=torch.float64, device=cdev)
    if dist:
        t_max = vals[0:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        sums = vals[1:].clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        elapsed, rays, samples = float(t_max[0]), float(sums[0]), float(sums[1])
        everyone = [torch.zeros_like(per_rank) for _ in range(world)]
        dist.all_gather(everyone, per_rank)
        rank_rows = [[float(x) for x in t.cpu()] for t in everyone]
    else:
        rays, samples = float(st["rays"]), float(st["samples"])
        rank_rows = [[float(x) for x in per_rank.cpu()]]
    collective = {"backend": dist.get_backend() if dist else None, "world": dist.get_world_size() if dist else 1,
                  "rehearsal": bool(args.rehearse),
                  "gather_ms": round(rank_rows[0][1], 3),  # rank 0: copy + gather + un-permute, per step
                  "gather_ms_per_rank": [round(x[1], 3) for x in rank_rows],
                  "rank_ms": [round(x[0], 3) for x in rank_rows],  # each rank's timed wall time per step
                  "rank_max_over_mean": round(max(x[0] for x in rank_rows) / (sum(x[0] for x in rank_rows) / len(rank_rows)), 4)}

    # standalone wf_trace launches for the roofline (outside the timed region): the same frame-group
    # workload as one timed launch (frames per group = F / (batches x 2)), run as ONE group
    # (RT_FLAG_SERIAL), so no other kernel shares the CUs; HIP events on the launch stream
    probe = None
    if st["trace_launches"]:
        from rtamd.renderer import RT_FLAG_SERIAL
        # (rt_stats.launches counts the batches a render call is split into; two frame groups each)
        per_group = max(1, -(-F * steps // (2 * max(1, st["launches"]))))
        r.reset_stats()
        r.render(cf.frame_params(W, H, flags=RT_FLAG_SERIAL), ro[-1 - per_group:-1])
        probe = r.stats()
        probe["frames"] = per_group

    frame_sha = None
    if args.frame_sha and rank == 0 and frame is not None and not args.no_gather:
        import hashlib
        torch.cuda.synchronize()
        frame_sha = hashlib.sha256(frame.cpu().numpy().tobytes()).hexdigest()

    # the reference's usage pattern (main.cpp:165-200): one frame per draw, outside the timed
    # region; throughput of back-to-back single-frame calls and the latency of a synchronised one
    base = (warm + steps) * F
    single = {}
    if n_single > 0:
        # back-to-back one-frame calls, one call in flight at a time and then with frames in flight
        # across calls (rt_set_pipeline: the GL driver's own frame queue; results unchanged)
        for depth in (args.pipeline, 1) if args.pipeline > 1 else (1,):
            r.set_pipeline(depth)
            # longest-first work order from one probe frame (rt_order_work; results unchanged): the
            # costliest 64-pixel blocks are queued first, so a one-frame pass ends on cheap blocks
            r.order_work(fp, ro[base:base + 1])
            r.render_async(fp, ro[base:base + 1])
            r.synchronize()
            t1 = time.perf_counter()
            for k in range(n_single):
                r.render_async(fp, ro[base + k:base + k + 1])
            r.synchronize()
            ms = round((time.perf_counter() - t1) * 1e3 / n_single, 3)
            single["ms_per_frame_single" if depth > 1 or args.pipeline <= 1 else "ms_per_frame_single_one_in_flight"] = ms
        single["single_frame_pipeline"] = max(1, args.pipeline)
        lat = []  # the median of as many synchronised calls as single frames (per-frame spread ~+-5%)
        for k in range(n_single):
            t2 = time.perf_counter()
            r.render_async(fp, ro[base + k:base + k + 1])
            r.synchronize()
            lat.append(time.perf_counter() - t2)
        single["ms_single_frame_latency"] = round(float(np.median(lat)) * 1e3, 3)

    # own-traversal visit counts (one extra frame, outside the timed region; tools/summarize_profile.py
    # drops the launches from this frame on)
    r.reset_stats()
    r.render(cf.frame_params(W, H, flags=RT_FLAG_COUNT_VISITS), ro[-1:])
    vis = r.stats()

    if rank != 0:
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return 0

    launch_ms = st["kernel_ms"] / max(1, st["launches"])                 # one render call (all passes)
    trace_ms = st["trace_ms"] / max(1, st["trace_launches"])              # wf_trace, per launch (HIP events)
    out = {
        "metric": METRIC,
        "value": round(rays / elapsed / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warm,
        "ms_per_step": round(elapsed * 1e3 / steps, 3),
        "ms_per_frame": round(elapsed * 1e3 / (steps * F), 4),
        **single,
        "msamples_per_s": round(samples / elapsed / 1e6, 2),
        "rays_per_sample": round(rays / max(1.0, samples), 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "reference scene assets (loong_100000.obj, floor.obj, peppermint_powerplant_1k.hdr); "
                "randOrigin from glibc srand(20221002) (in-tree restatement of rand())",
        "config": {"workload": f"{cfg.name}: {cfg.note}; {W}x{H}, maxBounce 8, BSDF+MIS+env",
                   "width": W, "height": H, "frames_per_step": F, "spp_timed": steps * F,
                   "tile": args.tile, "path_slots_per_rank": path_slots,
                   "parallelism": f"pixel-tiles x{world} + frame-end gather",
                   "tile_assignment": "cost-balanced (rt_tile_costs probe frame)" if balanced else "interleaved t % N",
                   "steps_in_flight": args.pipeline if pipelined else 1,
                   "triangles": sd.counts["n_triangles"], "bvh_nodes": sd.counts["n_nodes"]},
        "kernel": {"name": "wf_trace", "launches": st["trace_launches"],
                   "render_call_ms": round(launch_ms, 4), "render_calls": st["launches"],
                   # two frame groups on two streams: their launches overlap, so per-launch durations
                   # measured co-running add up to more than the step; the union of the launches'
                   # intervals is the time during which any traversal ran
                   "corunning_avg_launch_ms": round(trace_ms, 4),
                   "busy_ms_per_step": round(st.get("trace_busy_ms", 0.0) / max(1, steps), 3),
                   "busy_share_of_step": round(st.get("trace_busy_ms", 0.0) / max(1e-9, elapsed * 1e3), 4)},
        "collective": collective,
        "parity": "bit-exact vs oracle (tests/test_gpu_parity.py)",
    }
    if frame_sha:
        out["frame_sha256"] = frame_sha
    if args.rehearse:
        out["rehearsal"] = "all ranks on one GPU, gloo collectives (not a scaling measurement)"
    if vis["rays"]:
        out["own_traversal_per_ray"] = {"internal": round(vis["internal_pops"] / vis["rays"], 2),
                                        "leaf": round(vis["leaf_pops"] / vis["rays"], 2),
                                        "tri": round(vis["tri_tests"] / vis["rays"], 2)}

    # CPU baseline (rank 0, N = 1 only) and the §8(d) per-ray figure from its counters
    cnt = None
    if world == 1 and args.cpu_seconds > 0:
        out["cpu_baseline"], cnt = cpu_baseline(sd, env, W, H, fp, args.cpu_seconds, args.cpu_threads)
    prof = load_profile(args.config, W, H, F, path_slots)
    out["roofline"] = roofline(st, vis, cnt, prof, probe, steps)
    print(json.dumps(out), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
