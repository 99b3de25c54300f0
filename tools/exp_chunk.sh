#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/chunk
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/chunk/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/chunk/parity.log; exit 1; }
tail -1 gpurun_out/chunk/parity.log
for c in 64 128 256 512 1024; do
  RT_POOL_CHUNK=$c timeout -k 10 200 python3 tools/quick_perf.py --frames 32 --per-launch 16 > gpurun_out/chunk/c$c.log 2>&1 || exit 1
  echo "chunk $c: $(grep ms/frame gpurun_out/chunk/c$c.log)"
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/chunk/kt -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 16 > gpurun_out/chunk/kt.log 2>&1 || exit 1
python3 tools/pass_profile.py gpurun_out/chunk/kt/run_kernel_trace.csv | sed -n 4,6p
