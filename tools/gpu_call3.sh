# rebuilt internal levels (default) vs the reference's own: visits per ray, A/B, parity tests
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 0; do RT_REBUILD=$v timeout -k 10 200 python3 tools/quick_perf.py --frames 64 --per-launch 64 --count-frames 8 2>&1 | grep -E "ms/frame|visits" | sed "s/^/rebuild=$v /"; done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest3.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest3.log; exit 1; }
tail -1 gpurun_out/pytest3.log
timeout -k 10 500 python3 tools/ab_proc.py --whole --rounds 3 reb=default ref=default:RT_REBUILD=0 > gpurun_out/ab3.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab3.log; exit 1; }
tail -3 gpurun_out/ab3.log
