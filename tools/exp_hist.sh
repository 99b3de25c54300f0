#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hist
mkdir -p $O
RT_DEBUG_PASSES=1 timeout -k 10 200 python3 tools/quick_perf.py --frames 1 --per-launch 1 > $O/passes.log 2>&1 || { tail -5 $O/passes.log; exit 1; }
grep -A5 "group 0 pass" $O/passes.log | grep "pass\|steps/ray" | tail -60
