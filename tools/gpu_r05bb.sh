#!/bin/bash
# round 5: paths per thread of the camera-pass shade (CAM) 8 / 6 / 4: record parity on 6 and 4, C3 bulk A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bb; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
for v in sc6 sc4; do
  RTAMD_LIB=$E/librtamd_$v.so timeout -k 10 300 python3 -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k camera_hit_records > $O/rec_$v.log 2>&1 || { echo "$v record tests failed"; tail -20 $O/rec_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/rec_$v.log)"
done
bash tools/gpu_ab.sh r05bb_ab sc8=sc8 sc6=sc6 sc4=sc4
