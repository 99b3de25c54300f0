#!/bin/bash
# Per-pass kernel durations, one frame group (serial passes), 161 frames per launch.
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pp/kt -o run -- python3 tools/quick_perf.py --frames 161 --per-launch 161 > gpurun_out/pp/kt.log 2>&1 || exit 1
grep ms/frame gpurun_out/pp/kt.log
python3 tools/pass_profile.py gpurun_out/pp/kt/run_kernel_trace.csv | tail -3
