#!/bin/bash
# GPU parity tests on a variant library (RTAMD_LIB; dev-lib tests get RT_FAST_TRACE=1), then a
# process-per-measurement A/B of head vs that variant on C3 (whole 1024-frame steps) and C4.
#   gpurun -- bash tools/ab_fast.sh <tag> <variant.so>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-fast}
VAR=${2:-opengl-ray-tracing-framework_amd/lib/exp/librtamd_fast.so}
O=gpurun_out/$TAG
mkdir -p $O
RTAMD_LIB=$PWD/$VAR RT_FAST_TRACE=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ${TESTS:-} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
HEAD_SO=opengl-ray-tracing-framework_amd/lib/exp/librtamd_head.so
timeout -k 10 900 python3 tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds ${ROUNDS:-3} head=$HEAD_SO new=$VAR > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -3 $O/ab.log
timeout -k 10 600 python3 tools/ab_proc.py --config C4 --frames 256 --reps 2 --rounds 2 head=$HEAD_SO new=$VAR > $O/ab4.log 2>&1 || { tail -20 $O/ab4.log; exit 1; }
tail -3 $O/ab4.log
