#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/bpc
for b in 1 2 3 4 6; do
  RT_TRACE_BPC=$b timeout -k 10 200 python3 tools/quick_perf.py --frames 16 --per-launch 16 > gpurun_out/bpc/b$b.log 2>&1 || exit 1
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bpc/kt1 -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 16 > gpurun_out/bpc/kt1.log 2>&1 || exit 1
echo ok
