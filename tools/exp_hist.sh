#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/hist
mkdir -p $O
RT_DEBUG_PASSES=1 timeout -k 10 300 python3 tools/quick_perf.py --frames 1 --per-launch 1 --count-frames ${CF:-64} > $O/passes.log 2>&1 || { tail -5 $O/passes.log; exit 1; }
awk '/cum internal [1-9]/{p=1} p' $O/passes.log | grep "pass\|overflow\|steps/ray" | tail -80
