#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/quick
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/quick/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/quick/parity.log; exit 1; }
tail -1 gpurun_out/quick/parity.log
timeout -k 10 200 python3 tools/quick_perf.py --frames 32 --per-launch 16 > gpurun_out/quick/perf.log 2>&1 || exit 1
grep ms/frame gpurun_out/quick/perf.log
RT_GROUPS=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/quick/kt1 -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 16 > gpurun_out/quick/kt1.log 2>&1 || exit 1
python3 tools/pass_profile.py gpurun_out/quick/kt1/run_kernel_trace.csv | sed -n 1,6p
