#!/bin/bash
# GPU suite + default bench on the current build (round 5 checkpoint)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/chk2; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'], d['ms_per_frame'], d['ms_single_frame_latency'], d['ms_per_frame_single'], d['roofline']['frac'])"
