#!/bin/bash
# round 5: GPU suite after stripping the dead claim / statistics / culling-limit alternatives
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ba; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
