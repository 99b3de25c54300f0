#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
X=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_materials.py tests/test_gpu_cull.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python3 tools/ab_single.py --rounds 3 ${VARS:-help=default nohelp=$X/librtamd_nohelp.so} > $O/ab_single.log 2>&1 || { tail -20 $O/ab_single.log; exit 1; }
tail -6 $O/ab_single.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 1 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 tools/single_timeline.py $O/tr/run_kernel_trace.csv --calls 3 > $O/timeline.txt || exit 1
