#!/bin/bash
# One GPU call: the GPU test suite (verbose, per-test timeout), then the driver's default bench.
#   gpurun -- bash tools/gpu_check.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-chk}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${TESTS:-} > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; grep -E "FAILED|Error|error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
