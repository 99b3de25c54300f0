#!/bin/bash
# round 5: one-frame calls: per-group camera kernels (no cross-stream wait after wf_camera), head share
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_cpg.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py > $O/tests_cpg.log 2>&1 || { echo "cpg tests failed"; tail -20 $O/tests_cpg.log; exit 1; }
tail -1 $O/tests_cpg.log
V=""
for n in base15 cpg cpgh8 cpgh3 h8; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds 3 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -6 $O/single.log
