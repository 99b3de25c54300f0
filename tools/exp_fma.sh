# NEE light table: parity tests + bulk and C4 A/B against the HEAD build (development aid)
set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/fma
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_fullsize.py tests/test_gpu_materials.py tests/test_gpu_cull.py tests/test_interactive.py tests/test_display.py > gpurun_out/fma/tests.log 2>&1 || { tail -30 gpurun_out/fma/tests.log; exit 1; }
tail -2 gpurun_out/fma/tests.log
timeout -k 10 900 python3 tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 head=opengl-ray-tracing-framework_amd/lib/exp/librtamd_head.so fma=default > gpurun_out/fma/ab.log 2>&1
tail -3 gpurun_out/fma/ab.log
timeout -k 10 600 python3 tools/ab_proc.py --config C4 --frames 256 --reps 2 --rounds 2 head=opengl-ray-tracing-framework_amd/lib/exp/librtamd_head.so fma=default > gpurun_out/fma/ab4.log 2>&1
tail -3 gpurun_out/fma/ab4.log
