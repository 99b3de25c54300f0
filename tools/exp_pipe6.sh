# pipelined one-frame calls after the idle check: work-order dealing A/B (development aid)
set -e
cd /root/repo
mkdir -p gpurun_out/pipe6
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_api.py -k "pipelined or longest" tests/test_interactive.py > gpurun_out/pipe6/tests.log 2>&1
tail -2 gpurun_out/pipe6/tests.log
for c in C3 C4; do
timeout -k 10 600 python3 tools/ab_single.py --config $c --rounds 2 one=default:RT_AB_ORDER=1 two=default:RT_AB_ORDER=1,RT_AB_PIPE=2 \
  two_r1=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_ORDER_RANGES=1 two_np=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_PIX_SPLIT=0 > gpurun_out/pipe6/$c.log 2>&1
echo "== $c"; tail -4 gpurun_out/pipe6/$c.log
done
