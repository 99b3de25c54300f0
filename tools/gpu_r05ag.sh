#!/bin/bash
# round 5: N=8 rank shares: tile size of the balanced map; one frame group per rank launch
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ag; mkdir -p $O
for t in 16 32 64; do
  timeout -k 10 400 python3 tools/rank_sim.py --worlds 8 --assign balanced --reps 2 --tile $t --out $O/tile$t.jsonl > $O/tile$t.log 2>&1 || { tail -5 $O/tile$t.log; exit 1; }
  python3 -c "import sys,json; [print('tile $t', d['world'], d['max_ms'], d['mean_ms'], d['imbalance']) for d in map(json.loads, open(sys.argv[1]))]" $O/tile$t.jsonl
done
WORLDS=8 bash tools/rank_ab.sh r05ag_rank "- RT_GROUPS=1"
