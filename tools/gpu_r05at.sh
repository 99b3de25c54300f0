#!/bin/bash
# round 5, camera-record build: C4/C5 profiles + bench lines, C2 bench line, N=8 rank shares
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05at; mkdir -p $O
bash tools/profile_configs.sh r05 || exit 1
timeout -k 10 600 python3 bench.py --config C2 --frames-per-step 256 --steps 3 --warmup 1 > $O/bench_C2.json 2> $O/bench_C2.err || { echo "bench C2 failed"; tail $O/bench_C2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_C2.json'));print('C2', d['value'], d['ms_per_frame'], d.get('ms_single_frame_latency'))"
timeout -k 10 400 python3 tools/rank_sim.py --worlds 1,8 --assign balanced --reps 3 --tile 16 --out $O/rank.jsonl > $O/rank.log 2>&1 || { tail -5 $O/rank.log; exit 1; }
python3 -c "import sys,json; [print('rank', d['world'], d['max_ms'], d['mean_ms'], d['imbalance'], d.get('efficiency_vs_n1')) for d in map(json.loads, open(sys.argv[1]))]" $O/rank.jsonl
