#!/bin/bash
# N=8 per-rank shares on one GPU under several env settings (development aid)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/rank8
mkdir -p $O
for cfg in $CFGS; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $(echo $e | tr ',' ' ') timeout -k 10 300 python3 tools/rank_sim.py --worlds 1,8 --assign balanced > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "== $n: $(grep '"world": 8' $O/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['max_ms'], d['efficiency_vs_n1'], d['imbalance'])") N1: $(grep '"world": 1' $O/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['max_ms'])")"
done
