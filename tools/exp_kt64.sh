#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/kt64
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt64/kt -o run -- python3 tools/quick_perf.py --frames 64 --per-launch 64 > gpurun_out/kt64/kt.log 2>&1 || exit 1
