#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/quick
timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q -m gpu > gpurun_out/quick/parity.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/quick/parity.log; exit 1; }
tail -1 gpurun_out/quick/parity.log
timeout -k 10 300 python3 tools/quick_perf.py --frames 128 --per-launch 64 > gpurun_out/quick/perf.log 2>&1 || exit 1
grep ms/frame gpurun_out/quick/perf.log
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/quick/kt64 -o run -- python3 tools/quick_perf.py --frames 64 --per-launch 64 > gpurun_out/quick/kt64.log 2>&1 || exit 1
python3 tools/pass_profile.py gpurun_out/quick/kt64/run_kernel_trace.csv | sed -n 4,6p
