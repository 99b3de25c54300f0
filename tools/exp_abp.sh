#!/bin/bash
# Parity of the default build, process-level A/B of variants (AB="name=path ..."), then the
# per-pass profile (one frame group, 161 frames) of the default build.
export TMPDIR=/tmp
O=gpurun_out/abp
mkdir -p $O
[ -n "$SKIP_PARITY" ] || { timeout -k 10 400 python3 -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q -m gpu > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }; tail -1 $O/parity.log; }
timeout -k 10 600 python3 tools/ab_proc.py --rounds ${ROUNDS:-3} $ABOPT $AB > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
tail -${NV:-3} $O/ab.log
[ -n "$SKIP_PASSES" ] && exit 0
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/quick_perf.py --frames 161 --per-launch 161 > $O/kt.log 2>&1 || exit 1
python3 tools/pass_profile.py $O/kt/run_kernel_trace.csv | sed -n 4,6p
