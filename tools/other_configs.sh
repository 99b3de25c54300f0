# bench lines of the other configurations (C2, C4, C5: 256-frame steps) on the current build
set -e
cd /root/repo
for c in C2 C4 C5; do timeout -k 10 300 python3 bench.py --config $c --frames-per-step 256 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail gpurun_out/bench_$c.err; exit 1; }; python3 -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['ms_per_frame'], d.get('ms_per_frame_single'), d.get('ms_per_frame_single_one_in_flight'), d.get('ms_single_frame_latency'), d['rays_per_sample'], d['own_traversal_per_ray'])"; done
