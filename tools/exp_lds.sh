#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/lds
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/lds/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/lds/parity.log; exit 1; }
tail -1 gpurun_out/lds/parity.log
for k in 8 12 16 20 24; do
  RT_LDS_STACK=$k RT_DEBUG=1 timeout -k 10 300 python3 tools/quick_perf.py --frames 128 --per-launch 64 > gpurun_out/lds/k$k.log 2>&1 || exit 1
  echo "lds $k: $(grep ms/frame gpurun_out/lds/k$k.log) $(grep 'trace: lds' gpurun_out/lds/k$k.log | sed 's/.*occupancy API/occ/')"
done
