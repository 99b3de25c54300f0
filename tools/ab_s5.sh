# packed per-path seed/bounce/flags: parity (incl. staged start) + A/B against the 16-B layout
export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_s5.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_s5.log; exit 1; }
tail -1 gpurun_out/pytest_s5.log
RT_STAGES=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "config_matches" --timeout 300 --timeout-method thread > gpurun_out/pytest_s5s.log 2>&1 || { echo "staged tests failed"; tail -30 gpurun_out/pytest_s5s.log; exit 1; }
tail -1 gpurun_out/pytest_s5s.log
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 pack=default old=$L/librtamd_old.so > gpurun_out/ab_s5.log 2>&1 || { echo ab failed; exit 1; }
tail -3 gpurun_out/ab_s5.log
