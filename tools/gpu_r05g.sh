#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 1000 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 2 \
  base=$E/librtamd_devbase.so alt=$E/librtamd_altdev.so alt7=$E/librtamd_altdev.so:RT_TRACE_BPC=7 alt6=$E/librtamd_altdev.so:RT_TRACE_BPC=6 base6=$E/librtamd_devbase.so:RT_TRACE_BPC=6 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -7 $O/ab.log
# one-frame call timeline (rocprofv3 kernel trace of synchronised calls)
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 tools/single_calls.py --calls 8 > $O/tl.log 2>&1 || { echo "timeline failed"; tail -5 $O/tl.log; exit 1; }
python3 tools/single_timeline.py $(ls $O/tl/*/run_kernel_trace.csv $O/tl/run_kernel_trace.csv 2>/dev/null | head -1) --calls 3 > $O/timeline.txt 2>&1
tail -40 $O/timeline.txt
