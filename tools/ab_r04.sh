#!/bin/bash
# Round-4 development run (GPU box): checked fast-trace build on the small bench, the GPU tests on
# the fast variant, then bulk and one-frame A/Bs against the committed build.  Logs: gpurun_out/$TAG
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-r04}
O=gpurun_out/$TAG
mkdir -p $O
EXP=opengl-ray-tracing-framework_amd/lib/exp
DEV=opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
if [ -z "$SKIP_CHK" ]; then
  bash tools/chk_fast.sh > $O/chk.log 2>&1; tail -4 $O/chk.log
  grep -q "rc=0" $O/chk.log || { echo "check run failed"; exit 1; }
  if grep -q "rt check" $O/chk.log; then echo "bounds check fired"; exit 1; fi
fi
if [ -z "$SKIP_TESTS" ]; then
  RTAMD_LIB=$PWD/$EXP/librtamd_fastrel.so RT_FAST_TRACE=1 RT_FINISH_ROUNDS=3 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
[ -z "$SKIP_VISITS" ] && for F in 0 1; do  # visit counts per ray of the exact and the fast traversal (C3 1080p, 4 frames)
  RTAMD_LIB=$PWD/$DEV RT_FAST_TRACE=$F RT_ORD_KEY=${ORD:-centre} timeout -k 10 300 python3 tools/quick_perf.py --frames 4 --count-frames 4 2>&1 | tail -1 | sed "s/^/fast=$F /"
  RTAMD_LIB=$PWD/$DEV RT_FAST_TRACE=$F RT_ORD_KEY=corner timeout -k 10 300 python3 tools/quick_perf.py --frames 4 --count-frames 4 2>&1 | tail -1 | sed "s/^/fast=$F corner /"
done | tee $O/visits.log
timeout -k 10 1200 python3 tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds ${ROUNDS:-3} head=$EXP/librtamd_head.so \
  exact=$DEV:RT_FAST_TRACE=0 fast=$DEV:RT_FAST_TRACE=1 defer=$EXP/librtamd_fastdefer.so \
  corner=$DEV:RT_FAST_TRACE=1,RT_ORD_KEY=corner kl10=$DEV:RT_FAST_TRACE=1,RT_LDS_STACK=10 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -7 $O/ab.log
timeout -k 10 900 python3 tools/ab_single.py --config C3 --rounds 3 head=$EXP/librtamd_head.so:RT_AB_ORDER=1 \
  r1=$DEV:RT_AB_ORDER=1,RT_FINISH_ROUNDS=1,RT_FAST_TRACE=1 r3=$DEV:RT_AB_ORDER=1,RT_FINISH_ROUNDS=3,RT_FAST_TRACE=1 \
  ff=$EXP/librtamd_finfast.so:RT_AB_ORDER=1 \
  > $O/ab_single.log 2>&1 || { tail -20 $O/ab_single.log; exit 1; }
tail -4 $O/ab_single.log
