#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_emptyslot_r04.so timeout -k 10 300 python3 -u -m pytest -s -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "zero_direction and bulk" > $O/emptyslot.log 2>&1
rc=$?
echo "emptyslot rc=$rc"
grep -a "rt check" $O/emptyslot.log | sort | uniq -c | sort -rn | head -5
if [ $rc -ge 124 ]; then echo "stopping: rc $rc"; exit 1; fi
RT_DEBUG_PASSES=1 RT_GROUPS=1 timeout -k 10 300 python3 -u tools/pass_counts.py --config C3 --frames 64 > $O/passes_time.log 2>&1 || { echo "pass timing failed"; tail -5 $O/passes_time.log; exit 1; }
RT_DEBUG_PASSES=1 RT_GROUPS=1 timeout -k 10 300 python3 -u tools/pass_counts.py --config C3 --frames 64 --count > $O/passes_count.log 2>&1 || { echo "pass count failed"; tail -5 $O/passes_count.log; exit 1; }
RT_DEBUG_PASSES=1 RT_GROUPS=1 timeout -k 10 300 python3 -u tools/pass_counts.py --config C4 --frames 32 --count > $O/passes_count_C4.log 2>&1 || { echo "pass count C4 failed"; tail -5 $O/passes_count_C4.log; exit 1; }
grep -a "pass\|lane util" $O/passes_time.log | head -30
