#!/bin/bash
# round 5: tile size 16 vs 32 at N=1 and N=8 (interleaved, rank_sim)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ah; mkdir -p $O
for r in 1 2; do
for t in 32 16; do
  timeout -k 10 400 python3 tools/rank_sim.py --worlds 1,8 --assign balanced --reps 2 --tile $t --out $O/tile${t}_$r.jsonl > $O/tile${t}_$r.log 2>&1 || { tail -5 $O/tile${t}_$r.log; exit 1; }
  python3 -c "import sys,json; [print('tile $t', d['world'], d['max_ms'], d['mean_ms'], d['imbalance'], d['efficiency_vs_n1']) for d in map(json.loads, open(sys.argv[1]))]" $O/tile${t}_$r.jsonl
done
done
