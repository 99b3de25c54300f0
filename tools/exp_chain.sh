# chained batches: parity tests + bulk A/B (development aid)
set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/chain
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_api.py tests/test_gpu_fullsize.py > gpurun_out/chain/tests.log 2>&1
tail -2 gpurun_out/chain/tests.log
timeout -k 10 900 python3 tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 nochain=default:RT_BATCH_CHAIN=0 chain=default > gpurun_out/chain/ab.log 2>&1
tail -4 gpurun_out/chain/ab.log
