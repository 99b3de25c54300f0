#!/bin/bash
# round 5: the camera-record assumption checked on the GPU: an RT_CHECK build (which prints any
# frame whose trace result differs from its pixel's record) over the record and bench-shape tests
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ay; mkdir -p $O
RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_check.so timeout -k 10 500 python3 -u -m pytest -s -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_api.py -k "camera_hit_records or operating_point" > $O/check.log 2>&1
rc=$?
echo "rc=$rc"
grep -E 'PASSED|FAILED' $O/check.log | tail -8
echo "rt check lines: $(grep -c '\[rt check\]' $O/check.log)"
