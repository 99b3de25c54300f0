export TMPDIR=/tmp
mkdir -p gpurun_out/pp
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pp/t -o run -- python3 tools/quick_perf.py --frames 320 --per-launch 160 > gpurun_out/pp/qp.log 2>&1 || { echo fail; tail gpurun_out/pp/qp.log; exit 1; }
cat gpurun_out/pp/qp.log
f=$(find gpurun_out/pp/t -name '*kernel_trace.csv' | head -1)
python3 tools/pass_profile.py $f | tail -8
RT_GROUPS=1 RT_DEBUG_PASSES=1 timeout -k 10 300 python3 tools/quick_perf.py --frames 1 --count-frames 32 > gpurun_out/pp/dbg.log 2>&1 || { echo fail2; tail gpurun_out/pp/dbg.log; exit 1; }
grep -E "pass|lane" gpurun_out/pp/dbg.log | tail -30
