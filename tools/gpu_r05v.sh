#!/bin/bash
# round 5: one-frame call timeline on the current build (rocprofv3 kernel trace of synchronised calls)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 tools/single_calls.py --calls 8 > $O/tl.log 2>&1 || { echo "timeline failed"; tail -5 $O/tl.log; exit 1; }
python3 tools/single_timeline.py $(ls $O/tl/*/run_kernel_trace.csv $O/tl/run_kernel_trace.csv 2>/dev/null | head -1) --calls 3 > $O/timeline.txt 2>&1
tail -40 $O/timeline.txt
