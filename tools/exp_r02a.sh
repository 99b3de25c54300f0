#!/bin/bash
# r02 measurements: hardware-transcendental A/B (C3, C4), every rank's share at N = 1/2/4/8,
# and the per-pass kernel times of single-frame render calls (the reference's usage pattern).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
HW=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_hwmath.so
timeout -k 10 300 python3 tools/ab_proc.py --rounds 3 --whole base=default hw=$HW > $O/ab_hw_C3.log 2>&1 || { tail -20 $O/ab_hw_C3.log; exit 1; }
tail -3 $O/ab_hw_C3.log
timeout -k 10 300 python3 tools/ab_proc.py --config C4 --frames 256 --rounds 3 --whole base=default hw=$HW > $O/ab_hw_C4.log 2>&1 || { tail -20 $O/ab_hw_C4.log; exit 1; }
tail -3 $O/ab_hw_C4.log
timeout -k 10 300 python3 tools/rank_sim.py --out $O/rank_sim_C3.jsonl > $O/rank_sim.log 2>&1 || { tail -20 $O/rank_sim.log; exit 1; }
cat $O/rank_sim_C3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/single -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 1 > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
python3 tools/pass_profile.py $O/single/run_kernel_trace.csv | tail -6
