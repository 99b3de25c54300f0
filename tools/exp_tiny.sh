#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/tiny
for sz in 8 128 512; do
RT_GROUPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tiny/kt$sz -o run -- python3 tools/quick_perf.py --width $sz --height $sz --frames 4 --per-launch 4 > gpurun_out/tiny/t$sz.log 2>&1 || exit 1
done
echo ok
