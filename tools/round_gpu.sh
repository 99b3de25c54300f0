#!/bin/bash
# GPU tests + default bench line + rocprof evidence (run on the GPU box from the repo root)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
bash tools/profile_gpu.sh gpurun_out/prof || { echo "profile failed"; exit 1; }
