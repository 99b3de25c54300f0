#!/bin/bash
# single-frame call anatomy: rocprofv3 kernel timeline of one-frame calls + per-pass ray counts
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/single2
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 1 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 tools/single_timeline.py $O/tr/run_kernel_trace.csv --calls 2 > $O/timeline.txt || exit 1
cat $O/timeline.txt | head -120
RT_DEBUG_PASSES=1 timeout -k 10 200 python3 tools/quick_perf.py --frames 2 --per-launch 1 > $O/passes.log 2>&1 || { tail -5 $O/passes.log; exit 1; }
grep -v "4-wide" $O/passes.log | tail -60
