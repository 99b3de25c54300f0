#!/bin/bash
# round 5: segmented claims in the one-frame kernels (finisher, small passes); atomic throughput
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 60 tools/bin/atomic_bench > $O/atomics.log 2>&1 || { echo "atomic bench failed"; tail $O/atomics.log; exit 1; }
cat $O/atomics.log
RTAMD_LIB=$E/librtamd_fsseg.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py > $O/tests_fsseg.log 2>&1 || { echo "fsseg tests failed"; tail -20 $O/tests_fsseg.log; exit 1; }
tail -1 $O/tests_fsseg.log
V=""
for n in base13 fseg sseg fsseg; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 500 python3 -u tools/ab_single.py --config C3 --rounds 3 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -5 $O/single.log
