# pipelined batches: GPU parity tests + bench legs (development aid)
set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/pb2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_api.py tests/test_interactive.py tests/test_gpu_fullsize.py > gpurun_out/pb2/tests.log 2>&1
tail -3 gpurun_out/pb2/tests.log
timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --frames-per-step 256 --cpu-seconds 0 --single-frames 32 > gpurun_out/pb2/b256.json 2> gpurun_out/pb2/b256.err
timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --frames-per-step 256 --cpu-seconds 0 --single-frames 32 --pipeline-steps > gpurun_out/pb2/b256p.json 2> gpurun_out/pb2/b256p.err
python3 - <<'PY'
import json
for f in ("b256", "b256p"):
    d = json.loads(open(f"gpurun_out/pb2/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_frame"], d.get("ms_per_frame_single"), d.get("ms_per_frame_single_one_in_flight"), d.get("ms_single_frame_latency"), d["config"].get("steps_in_flight"))
PY
