#!/bin/bash
# GPU parity tests, then process-per-measurement A/B of the working tree's librtamd.so against the
# committed one (tools/build_head_variant.sh builds lib/exp/librtamd_head.so first, on the CPU side):
# C3 whole 1024-frame steps and C4 256-frame launches.  Development aid; logs under gpurun_out/$TAG.
#   bash tools/build_head_variant.sh && gpurun -- bash tools/ab_gpu.sh mytag
set -e
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-ab}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
HEAD_SO=opengl-ray-tracing-framework_amd/lib/exp/librtamd_head.so
timeout -k 10 900 python3 tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 head=$HEAD_SO new=default > $O/ab.log 2>&1
tail -3 $O/ab.log
timeout -k 10 600 python3 tools/ab_proc.py --config C4 --frames 256 --reps 2 --rounds 2 head=$HEAD_SO new=default > $O/ab4.log 2>&1
tail -3 $O/ab4.log
