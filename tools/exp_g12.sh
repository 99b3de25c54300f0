#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/g12
for g in 1 2; do
  RT_GROUPS=$g timeout -k 10 200 python3 tools/quick_perf.py --frames 32 --per-launch 16 > gpurun_out/g12/g$g.log 2>&1 || exit 1
  echo "groups $g: $(grep ms/frame gpurun_out/g12/g$g.log)"
done
RT_GROUPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/g12/kt -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 16 > gpurun_out/g12/kt.log 2>&1 || exit 1
