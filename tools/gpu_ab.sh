#!/bin/bash
# Process-per-measurement A/B of release-like variants on C3 whole 1024-frame steps (and C4 256-frame
# calls with C4=1):  gpurun -- bash tools/gpu_ab.sh <tag> name=lib/exp/librtamd_x.so ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
E=opengl-ray-tracing-framework_amd/lib/exp
ARGS=""
for v in "$@"; do ARGS="$ARGS ${v%%=*}=$PWD/$E/librtamd_${v#*=}.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds ${ROUNDS:-3} $ARGS > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -4 $O/ab.log
if [ -n "$C4" ]; then
  timeout -k 10 600 python3 -u tools/ab_proc.py --config C4 --frames 256 --reps 2 --rounds 2 $ARGS > $O/ab4.log 2>&1 || { tail -20 $O/ab4.log; exit 1; }
  tail -4 $O/ab4.log
fi
