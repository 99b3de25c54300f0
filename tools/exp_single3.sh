#!/bin/bash
# single-frame call timelines under several env settings (development aid)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/single3
mkdir -p $O
for cfg in $CFGS; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$n -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 1 > $O/tr_$n.log 2>&1 || { tail -5 $O/tr_$n.log; exit 1; }
  python3 tools/single_timeline.py $O/tr_$n/run_kernel_trace.csv --calls 6 > $O/timeline_$n.txt || exit 1
  echo "== $n: $(grep 'ms/frame' $O/tr_$n.log)"
  grep "^call\|mean span" $O/timeline_$n.txt
done
