#!/bin/bash
# round 5: shade sub-iterations for the bulk groups only (parity on the variant, bulk and one-frame A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_sb4.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py > $O/tests_sb4.log 2>&1 || { echo "sb4 tests failed"; tail -20 $O/tests_sb4.log; exit 1; }
tail -1 $O/tests_sb4.log
V=""
for n in base17 sb4 sb5 sb6; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -5 $O/bulk.log
timeout -k 10 400 python3 -u tools/ab_single.py --config C3 --rounds 2 base17=$E/librtamd_base17.so sb4=$E/librtamd_sb4.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -3 $O/single.log
