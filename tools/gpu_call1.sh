export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python3 tools/ab_proc.py --whole --rounds 3 base=default nosob=opengl-ray-tracing-framework_amd/lib/exp/librtamd_nosob.so > gpurun_out/ab1.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab1.log; exit 1; }
cat gpurun_out/ab1.log
