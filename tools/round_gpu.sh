#!/bin/bash
# Round evidence on the GPU box (repo root): GPU tests, rocprofv3 kernel trace + PMC passes of
# the bench workload, their summary into profiles/ (PMC traffic per wf_trace launch), then the
# driver's bench command (which reads that summary).  profiles/ comes back via gpurun_out/profiles.
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r05_C3}
mkdir -p gpurun_out/profiles
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
bash tools/profile_gpu.sh gpurun_out/prof || { echo "profile failed"; exit 1; }
python3 tools/summarize_profile.py gpurun_out/prof $TAG \
  '{"config": "C3", "width": 1920, "height": 1080, "frames_per_step": 1024, "path_slots_per_rank": 2139095040, "probe_trace_launches": 9, "command": "bash tools/profile_gpu.sh (bench.py --steps 3 --warmup 1 --cpu-seconds 0 --single-frames 0)"}' > gpurun_out/summary.log || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cp gpurun_out/bench.json gpurun_out/profiles/${TAG%_C3}_bench_C3.json
cp profiles/${TAG}_* profiles/pmc_C3.json gpurun_out/profiles/
[ -n "$SKIP_INTERACTIVE" ] && exit 0
timeout -k 10 300 python3 tools/interactive_demo.py --config C3 --frames 60 --out gpurun_out/interactive > gpurun_out/interactive.log 2>&1 || { echo "interactive failed"; tail -5 gpurun_out/interactive.log; exit 1; }
cp gpurun_out/interactive/C3_interactive.json gpurun_out/profiles/${TAG}_interactive.json
tail -7 gpurun_out/interactive.log
timeout -k 10 300 python3 tools/interactive_demo.py --config C3 --frames 60 --in-flight 2 --out gpurun_out/interactive2 > gpurun_out/interactive2.log 2>&1 || { echo "interactive (2 in flight) failed"; tail -5 gpurun_out/interactive2.log; exit 1; }
cp gpurun_out/interactive2/C3_interactive.json gpurun_out/profiles/${TAG}_interactive_in_flight2.json
tail -7 gpurun_out/interactive2.log
