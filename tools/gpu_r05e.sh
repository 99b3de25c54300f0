#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for cfg in C3 C4; do
  for sub in 0 1; do
    RT_SUBLEAF=$sub RT_DEBUG_PASSES=1 RT_GROUPS=1 timeout -k 10 300 python3 -u tools/pass_counts.py --config $cfg --frames 16 --count > $O/count_${cfg}_sub$sub.log 2>&1 || { echo "count failed"; tail -5 $O/count_${cfg}_sub$sub.log; exit 1; }
    tail -1 $O/count_${cfg}_sub$sub.log | cut -c1-200
  done
done
C4=1 bash tools/gpu_ab.sh r05e climit=r05climit sub=sub
