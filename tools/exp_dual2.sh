#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/dual2
for m in 2 3; do
RT_TRACE_MODE=$m RT_GROUPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dual2/kt$m -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 16 > gpurun_out/dual2/kt$m.log 2>&1 || exit 1
done
