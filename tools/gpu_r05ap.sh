#!/bin/bash
# round 5: the finisher takes over after pass 1's trace, starting with pass 1's shade steps (parity, one-frame A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ap; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_sfirst.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_sfirst.log 2>&1 || { echo "sfirst tests failed"; tail -30 $O/tests_sfirst.log; exit 1; }
tail -1 $O/tests_sfirst.log
timeout -k 10 500 python3 -u tools/ab_single.py --config C3 --rounds 4 base31=$E/librtamd_base31.so sfirst=$E/librtamd_sfirst.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -3 $O/single.log
