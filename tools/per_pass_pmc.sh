#!/bin/bash
# Per-launch PMC of one 256-frame C3 frame group (RT_GROUPS=1, dev library; dispatches serialised by
# the counter collection, so every duration is a standalone launch): FETCH_SIZE, WRITE_SIZE and the
# SQ issue counters of each wf_trace / wf_shade pass, then tools/per_pass_pmc.py's table.
#   gpurun -- bash tools/per_pass_pmc.sh [out dir]
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/ppmc}
mkdir -p $O
export RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
export RT_GROUPS=1
Q="tools/pass_counts.py --frames 256 --max-paths 530841600"
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/f -o run -- python3 $Q > $O/f.log 2>&1 || { echo "fetch pass failed"; tail -5 $O/f.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/w -o run -- python3 $Q > $O/w.log 2>&1 || { echo "write pass failed"; tail -5 $O/w.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/s -o run -- python3 $Q > $O/s.log 2>&1 || { echo "sq pass failed"; tail -5 $O/s.log; exit 1; }
python3 tools/per_pass_pmc.py $O
