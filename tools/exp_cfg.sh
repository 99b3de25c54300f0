#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/cfg
mkdir -p $O
for c in C3 C4; do
RT_DEBUG_PASSES=1 timeout -k 10 300 python3 tools/quick_perf.py --config $c --frames 1 --per-launch 1 --count-frames 32 > $O/$c.log 2>&1 || { tail -5 $O/$c.log; exit 1; }
echo "== $c"; awk '/cum internal [1-9]/{p=1} p' $O/$c.log | grep "group 0 pass\|lane util\|visits per ray" | head -30
done
