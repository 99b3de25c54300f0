#!/bin/bash
# round 5: non-temporal loads of the shade's and blend's read-once rows (GPU suite, C3 bulk and one-frame A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bc; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05bc_ab ntl0=ntl0 ntl1=ntl1 || exit 1
timeout -k 10 400 python3 -u tools/ab_single.py --config C3 --rounds 3 ntl0=$E/librtamd_ntl0.so ntl1=$E/librtamd_ntl1.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -3 $O/single.log
