# Evidence on the current build: GPU tests, one-frame A/B against lib/exp/librtamd_r3e.so (REV=<rev> NAME=r3e
# tools/build_head_variant.sh), the driver bench command and the other configurations.  Logs in gpurun_out/ev.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ev
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ev/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/ev/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/ev/pytest_gpu.log
timeout -k 10 300 python3 tools/ab_single.py --config C3 --rounds 3 prev=opengl-ray-tracing-framework_amd/lib/exp/librtamd_r3e.so new=default > gpurun_out/ev/single.log 2>&1 || exit 1
tail -3 gpurun_out/ev/single.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/ev/bench.json 2> gpurun_out/ev/bench.err || { tail -20 gpurun_out/ev/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ev/bench.json'));print(d['value'], d['ms_per_frame'], d['ms_single_frame_latency'], d['ms_per_frame_single'])"
for c in C2 C4 C5; do timeout -k 10 300 python3 bench.py --config $c --frames-per-step 256 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/ev/bench_$c.json 2> gpurun_out/ev/bench_$c.err || { tail gpurun_out/ev/bench_$c.err; exit 1; }; python3 -c "import json;d=json.load(open('gpurun_out/ev/bench_$c.json'));print('$c', d['value'], d['ms_per_frame'], d.get('ms_per_frame_single'), d.get('ms_single_frame_latency'), d['rays_per_sample'], d['own_traversal_per_ray'])"; done
