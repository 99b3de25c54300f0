export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest28.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest28.log; exit 1; }
tail -1 gpurun_out/pytest28.log
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 env1=default old=$L/librtamd_old.so > gpurun_out/ab28.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab28.log; exit 1; }
tail -3 gpurun_out/ab28.log
