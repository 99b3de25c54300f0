#!/bin/bash
# round 5: pass counters on lines of their own; finisher claim pools (parity on the combined variant, one-frame A/B, bulk A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_linesfp64.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py > $O/tests_linesfp64.log 2>&1 || { echo "linesfp64 tests failed"; tail -20 $O/tests_linesfp64.log; exit 1; }
tail -1 $O/tests_linesfp64.log
V=""
for n in base14 lines fp16 fp64 linesfp64; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds 3 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -6 $O/single.log
timeout -k 10 700 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 base14=$E/librtamd_base14.so lines=$E/librtamd_lines.so > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -3 $O/bulk.log
