#!/bin/bash
# round 5: top QNodes in LDS (5 / 21) for wf_trace (parity on the variant, bulk and one-frame A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ak; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_nc21.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py > $O/tests_nc21.log 2>&1 || { echo "nc21 tests failed"; tail -20 $O/tests_nc21.log; exit 1; }
tail -1 $O/tests_nc21.log
V=""
for n in base26 nc5 nc21; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -4 $O/bulk.log
timeout -k 10 500 python3 -u tools/ab_single.py --config C3 --rounds 3 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -4 $O/single.log
