# pipelined one-frame calls: parity tests, then A/B of the single-frame timing (development aid)
set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_api.py -k "pipelined or longest or progressive" > gpurun_out/pipe/tests.log 2>&1
tail -3 gpurun_out/pipe/tests.log
timeout -k 10 400 python3 tools/ab_single.py --rounds 2 base=default:RT_AB_ORDER=1 p2=default:RT_AB_ORDER=1,RT_AB_PIPE=2 p3=default:RT_AB_ORDER=1,RT_AB_PIPE=3 > gpurun_out/pipe/ab.log 2>&1
cat gpurun_out/pipe/ab.log
RT_AB_ORDER=1 RT_AB_PIPE=2 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pipe/prof -o run -- python3 tools/ab_single.py --one default --calls 24 > gpurun_out/pipe/prof.log 2>&1
f=$(find gpurun_out/pipe/prof -name '*kernel_trace.csv' | head -1)
python3 tools/single_timeline.py "$f" --calls 4 > gpurun_out/pipe/timeline.txt
tail -40 gpurun_out/pipe/timeline.txt
