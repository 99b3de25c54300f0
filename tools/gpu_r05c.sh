#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
MP=$((256*1920*1080))
RT_DEBUG_PASSES=1 RT_GROUPS=1 timeout -k 10 300 python3 -u tools/pass_counts.py --config C3 --frames 256 --max-paths $MP > $O/passes256_time.log 2>&1 || { echo "pass timing failed"; tail -5 $O/passes256_time.log; exit 1; }
grep -a "\] group" $O/passes256_time.log
RT_DEBUG_PASSES=1 RT_GROUPS=1 timeout -k 10 300 python3 -u tools/pass_counts.py --config C3 --frames 256 --max-paths $MP --count > $O/passes256_count.log 2>&1 || { echo "pass count failed"; tail -5 $O/passes256_count.log; exit 1; }
bash tools/gpu_ab.sh r05c base=r05base climit=climit
