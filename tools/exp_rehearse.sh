# multi-rank bench rehearsal on one GPU (development aid)
set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/reh
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bench_gpu.py > gpurun_out/reh/tests.log 2>&1 || { tail -40 gpurun_out/reh/tests.log; exit 1; }
tail -5 gpurun_out/reh/tests.log
