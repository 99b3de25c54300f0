#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h; mkdir -p $O
DEV=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 2 \
  base=$DEV st2=$DEV:RT_TRACE_STATIC_FROM=2 st4=$DEV:RT_TRACE_STATIC_FROM=4 st0=$DEV:RT_TRACE_STATIC_FROM=0 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -6 $O/ab.log
WORLDS=1,8 bash tools/rank_ab.sh r05h_rank "- RT_TRACE_STATIC_FROM=2 RT_TRACE_STATIC_FROM=0"
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_blendpf.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py > $O/blend_tests.log 2>&1 || { echo "blend tests failed"; tail -20 $O/blend_tests.log; exit 1; }
tail -1 $O/blend_tests.log
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 base=$E/librtamd_r05climit.so blendpf=$E/librtamd_blendpf.so > $O/ab_blend.log 2>&1 || { tail -20 $O/ab_blend.log; exit 1; }
tail -3 $O/ab_blend.log
