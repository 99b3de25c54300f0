#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/wlog
mkdir -p $O
RT_DEBUG_PASSES=1 RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_wlog.so timeout -k 10 200 python3 tools/quick_perf.py --frames 2 --per-launch 1 --count-frames 1 > $O/passes.log 2>&1 || { tail -5 $O/passes.log; exit 1; }
awk '/group 0 pass 0/{n++} n==2' $O/passes.log | grep "pass\|waves:" | head -40
