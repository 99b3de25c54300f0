#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/dual
RT_TRACE_MODE=3 timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/dual/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/dual/parity.log; exit 1; }
tail -1 gpurun_out/dual/parity.log
for m in 2 3; do
  RT_TRACE_MODE=$m timeout -k 10 200 python3 tools/quick_perf.py --frames 32 --per-launch 16 > gpurun_out/dual/m$m.log 2>&1 || exit 1
  echo "mode $m: $(grep ms/frame gpurun_out/dual/m$m.log)"
done
RT_TRACE_MODE=3 RT_GROUPS=1 RT_DEBUG_PASSES=1 timeout -k 10 200 python3 tools/quick_perf.py --frames 16 --per-launch 16 --flags 2 > gpurun_out/dual/count.log 2>&1 || exit 1
