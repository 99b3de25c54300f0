#!/bin/bash
# GPU tests (optional), then bulk A/B of VARIANTS (lib/exp/librtamd_<v>.so or name=default:ENV) on C3 (and C4 with C4=1)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab3
mkdir -p $O
X=$PWD/opengl-ray-tracing-framework_amd/lib/exp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
args=""
for v in $VARIANTS; do case $v in *=*) args="$args $v";; *) args="$args $v=$X/librtamd_$v.so";; esac; done
timeout -k 10 600 python3 tools/ab_proc.py --rounds ${ROUNDS:-3} --whole base=default $args > $O/ab_C3.log 2>&1 || { tail -20 $O/ab_C3.log; exit 1; }
tail -$((2 + $(echo $VARIANTS | wc -w))) $O/ab_C3.log
if [ -n "$C4" ]; then
  timeout -k 10 600 python3 tools/ab_proc.py --config C4 --frames 256 --rounds ${ROUNDS:-3} --whole base=default $args > $O/ab_C4.log 2>&1 || { tail -20 $O/ab_C4.log; exit 1; }
  tail -$((2 + $(echo $VARIANTS | wc -w))) $O/ab_C4.log
fi
