#!/bin/bash
# round 5: camera-pass shade fetches its block-iteration's trace results at once (parity, bulk, one-frame)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05af; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_camres.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py > $O/tests_camres.log 2>&1 || { echo "camres tests failed"; tail -20 $O/tests_camres.log; exit 1; }
tail -1 $O/tests_camres.log
timeout -k 10 700 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 base22=$E/librtamd_base22.so camres=$E/librtamd_camres.so > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -3 $O/bulk.log
timeout -k 10 400 python3 -u tools/ab_single.py --config C3 --rounds 3 base22=$E/librtamd_base22.so camres=$E/librtamd_camres.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -3 $O/single.log
