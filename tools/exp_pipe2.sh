# pipelined session + async display: parity tests, interactive timings (development aid)
set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe2
timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_interactive.py tests/test_gpu_api.py tests/test_display.py > gpurun_out/pipe2/tests.log 2>&1
tail -3 gpurun_out/pipe2/tests.log
timeout -k 10 200 python3 tools/interactive_demo.py --config C3 --frames 60 --out gpurun_out/pipe2/i1 > gpurun_out/pipe2/i1.log 2>&1
timeout -k 10 200 python3 tools/interactive_demo.py --config C3 --frames 60 --in-flight 2 --out gpurun_out/pipe2/i2 > gpurun_out/pipe2/i2.log 2>&1
timeout -k 10 200 python3 tools/interactive_demo.py --config C3 --frames 60 --in-flight 3 --out gpurun_out/pipe2/i3 > gpurun_out/pipe2/i3.log 2>&1
cat gpurun_out/pipe2/i1.log gpurun_out/pipe2/i2.log gpurun_out/pipe2/i3.log
