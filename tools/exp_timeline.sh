#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
RT_GROUPS=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl/kt -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 16 > gpurun_out/tl/kt.log 2>&1 || exit 1
echo ok
