#!/bin/bash
# round 5: camera-pass shade in its own instantiation with the V-only BSDF terms in the records
# (parity suite; negative control with poisoned V terms: the C3 bulk record cases must fail, the
# small-kernel case must pass; C3 bulk A/B against the previous build)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05as; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
RTAMD_LIB=$E/librtamd_poisonv.so timeout -k 10 300 python3 -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k camera_hit_records > $O/poison.log 2>&1
echo "poison rc=$?"
grep -E 'PASSED|FAILED' $O/poison.log | grep -v '^FAILED' | tail -6
bash tools/gpu_ab.sh r05as_ab crec1=crec1 camv=camv
