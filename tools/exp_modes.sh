#!/bin/bash
# A/B of the trace schedules x BVH width: parity, then C3 1080p timing (development aid)
export TMPDIR=/tmp
mkdir -p gpurun_out/modes
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/modes/parity.log 2>&1 || { echo "parity failed"; exit 1; }
for w in 2 4; do
  for m in 0 1 2; do
    RT_BVH_WIDTH=$w RT_TRACE_MODE=$m timeout -k 10 200 python3 tools/quick_perf.py --frames 16 --per-launch 4 > gpurun_out/modes/perf_w${w}_m${m}.log 2>&1 || exit 1
  done
done
RT_TRACE_MODE=1 timeout -k 10 200 python3 tools/quick_perf.py --frames 8 --per-launch 4 --flags 2 > gpurun_out/modes/count_w4.log 2>&1 || exit 1
echo ok
