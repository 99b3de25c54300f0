#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/passes
RT_GROUPS=1 RT_DEBUG_PASSES=1 timeout -k 10 200 python3 tools/quick_perf.py --frames 16 --per-launch 16 --flags 2 > gpurun_out/passes/count.log 2>&1 || exit 1
echo ok
