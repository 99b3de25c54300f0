export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest26.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest26.log; exit 1; }
tail -1 gpurun_out/pytest26.log
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pp26/t -o run -- python3 tools/quick_perf.py --frames 320 --per-launch 160 > gpurun_out/pp26.log 2>&1 || { echo fail; exit 1; }
f=$(find gpurun_out/pp26/t -name '*kernel_trace.csv' | head -1)
python3 tools/pass_profile.py $f | sed -n 4,6p
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 new=default old=$L/librtamd_old.so > gpurun_out/ab26.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab26.log; exit 1; }
tail -3 gpurun_out/ab26.log
