#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/stag
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/stag/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/stag/parity.log; exit 1; }
tail -1 gpurun_out/stag/parity.log
for g in 2 4; do for st in -1 1 2 3; do
  RT_GROUPS=$g RT_STAGGER=$st timeout -k 10 200 python3 tools/quick_perf.py --frames 32 --per-launch 16 > gpurun_out/stag/g${g}s${st}.log 2>&1 || exit 1
  echo "groups $g stagger $st: $(grep ms/frame gpurun_out/stag/g${g}s${st}.log)"
done; done
for st in 1 2; do
  RT_GROUPS=4 RT_STAGGER=$st timeout -k 10 200 python3 tools/quick_perf.py --frames 64 --per-launch 32 > gpurun_out/stag/g4s${st}f32.log 2>&1 || exit 1
  echo "groups 4 stagger $st 32 frames: $(grep ms/frame gpurun_out/stag/g4s${st}f32.log)"
done
