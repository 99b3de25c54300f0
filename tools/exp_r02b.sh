#!/bin/bash
# r02: GPU tests, per-rank balance (interleaved vs cost-balanced tile maps), quick bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python3 tools/rank_sim.py --out $O/rank_sim_C3.jsonl > $O/rank_sim.log 2>&1 || { tail -20 $O/rank_sim.log; exit 1; }
cat $O/rank_sim_C3.jsonl
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_frame'],d['ms_per_frame_single'])"
