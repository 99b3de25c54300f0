#!/bin/bash
# round 5: per-pixel camera-hit records in the bulk camera-pass shade (parity suite, C3 bulk A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aq; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_ab.sh r05aq_ab crec0=crec0 crec1=crec1
