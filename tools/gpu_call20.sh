export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$PWD/$L/librtamd_q1.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest20.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest20.log; exit 1; }
tail -1 gpurun_out/pytest20.log
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default q1=$L/librtamd_q1.so q2=$L/librtamd_q2.so > gpurun_out/ab20.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab20.log; exit 1; }
tail -4 gpurun_out/ab20.log
