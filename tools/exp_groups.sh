#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/groups
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/groups/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/groups/parity.log; exit 1; }
tail -1 gpurun_out/groups/parity.log
for g in 1 2 3 4; do
  RT_GROUPS=$g timeout -k 10 200 python3 tools/quick_perf.py --frames 32 --per-launch 16 > gpurun_out/groups/g$g.log 2>&1 || { echo "g$g failed"; exit 1; }
  echo "groups $g: $(grep ms/frame gpurun_out/groups/g$g.log)"
done
RT_GROUPS=4 RT_MAX_SLOTS=134217728 timeout -k 10 200 python3 tools/quick_perf.py --frames 64 --per-launch 32 > gpurun_out/groups/g4f32.log 2>&1 || exit 1
echo "groups 4, 32 frames: $(grep ms/frame gpurun_out/groups/g4f32.log)"
