# other configurations + full GPU suite on the current build
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest23.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest23.log; exit 1; }
tail -1 gpurun_out/pytest23.log
for c in C2 C3 C4 C5; do timeout -k 10 300 python3 bench.py --config $c --frames-per-step 256 --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail gpurun_out/bench_$c.err; exit 1; }; python3 -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));print('$c', d['value'], d['ms_per_frame'], d['rays_per_sample'], d['own_traversal_per_ray'])"; done
