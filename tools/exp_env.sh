#!/bin/bash
# A/B of runtime settings: ENVS="A=1 B=2" "C=3" ... each a set of env assignments (one bench + visits each)
export TMPDIR=/tmp
O=gpurun_out/env
mkdir -p $O
[ -n "$SKIP_PARITY" ] || timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
[ -n "$SKIP_PARITY" ] || tail -1 $O/parity.log
i=0
for e in "$@"; do
  i=$((i+1))
  env $e timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --cpu-seconds 0 > $O/bench_$i.log 2>&1 || exit 1
  echo "[$e] bench: $(python3 -c "import json;d=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_frame'],d['kernel']['avg_launch_ms'],d.get('own_traversal_per_ray'))")"
done
