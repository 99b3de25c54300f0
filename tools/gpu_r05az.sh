#!/bin/bash
# round 5: camera-record parity on the glass and jade scenes (bulk kernels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05az; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k camera_hit_records > $O/records.log 2>&1 || { echo "record tests failed"; tail -30 $O/records.log; exit 1; }
grep -E 'PASSED|FAILED|passed|failed' $O/records.log | tail -8
