# round evidence (tests, profiles, bench) + the other configurations
bash tools/round_gpu.sh || exit 1
for c in C2 C4 C5; do timeout -k 10 300 python3 bench.py --config $c --frames-per-step 256 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail gpurun_out/bench_$c.err; exit 1; }; python3 -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['ms_per_frame'], d['rays_per_sample'], d['own_traversal_per_ray'])"; done
