#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/fprof
mkdir -p $O
X=$PWD/opengl-ray-tracing-framework_amd/lib/exp
for v in fprof0 fprof; do
RT_FINISH_PROF=1 RTAMD_LIB=$X/librtamd_$v.so timeout -k 10 200 python3 tools/quick_perf.py --frames 3 --per-launch 1 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
echo "== $v"; grep "wf_finish\|wave" $O/$v.log | tail -18
done
