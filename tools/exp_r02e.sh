#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
X=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python3 tools/ab_single.py --rounds 3 head=$X/librtamd_head.so new=default sm4=$X/librtamd_sm4.so sm8=$X/librtamd_sm8.so sm32=$X/librtamd_sm32.so sm64=$X/librtamd_sm64.so p2=default:RT_FINISH_PASS=2 > $O/ab_single.log 2>&1 || { tail -20 $O/ab_single.log; exit 1; }
tail -8 $O/ab_single.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 1 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 tools/single_timeline.py $O/tr/run_kernel_trace.csv --calls 3 > $O/timeline.txt || exit 1
