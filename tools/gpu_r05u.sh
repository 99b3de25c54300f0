#!/bin/bash
# round 5: per-pass kernel durations of one 256-frame group (C3 1080p, one stream, no syncs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/shp -o run -- python3 tools/pass_counts.py --frames 256 --max-paths 530841600 > $O/run.log 2>&1 || { tail -20 $O/run.log; exit 1; }
python3 tools/pass_kernel_times.py $O/shp/run_kernel_trace.csv --last 24 > $O/times.txt
cat $O/times.txt
