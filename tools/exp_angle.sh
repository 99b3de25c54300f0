set -e
cd /root/repo
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_api.py -k "env_angle or pipelined" > gpurun_out/angle.log 2>&1 || { tail -30 gpurun_out/angle.log; exit 1; }
tail -2 gpurun_out/angle.log
