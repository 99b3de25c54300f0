#!/bin/bash
# Round-4 development run (GPU box): optionally the checked fast-trace build on the small bench and
# the GPU tests on the release-like fast variant, then bulk and one-frame A/Bs against the round-3
# build (lib/exp/librtamd_head.so from b704dc8).  Logs: gpurun_out/$TAG
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/$TAG
mkdir -p $O
EXP=opengl-ray-tracing-framework_amd/lib/exp
DEV=opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
# BULK / SINGLE may name the libraries as $DEV and $EXP/<file> (single-quoted by the caller)
BULK=${BULK//\$DEV/$DEV}; BULK=${BULK//\$EXP/$EXP}
SINGLE=${SINGLE//\$DEV/$DEV}; SINGLE=${SINGLE//\$EXP/$EXP}
if [ -n "$CHK" ]; then
  bash tools/chk_fast.sh > $O/chk.log 2>&1; tail -4 $O/chk.log
  grep -q "rc=0" $O/chk.log || { echo "check run failed"; exit 1; }
  if grep -q "rt check" $O/chk.log; then echo "bounds check fired"; exit 1; fi
fi
if [ -n "$TESTS" ]; then
  RTAMD_LIB=$PWD/$EXP/librtamd_fastrel.so RT_FAST_TRACE=1 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
if [ -n "$BULK" ]; then
  timeout -k 10 1500 python3 tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds ${ROUNDS:-3} head=$EXP/librtamd_head.so $BULK > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
  tail -$(( $(echo $BULK | wc -w) + 2 )) $O/ab.log
fi
if [ -n "$SINGLE" ]; then
  timeout -k 10 900 python3 tools/ab_single.py --config C3 --rounds 3 head=$EXP/librtamd_head.so:RT_AB_ORDER=1 $SINGLE > $O/ab_single.log 2>&1 || { tail -20 $O/ab_single.log; exit 1; }
  tail -$(( $(echo $SINGLE | wc -w) + 2 )) $O/ab_single.log
fi
