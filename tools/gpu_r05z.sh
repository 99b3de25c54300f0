#!/bin/bash
# round 5: bulk shade sub-iterations 6-8 (bulk A/B, N=8 rank shares)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base17 sb6 sb7 sb8; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -5 $O/bulk.log
for n in base17 sb8; do
  RTAMD_LIB=$E/librtamd_$n.so timeout -k 10 400 python3 tools/rank_sim.py --worlds 1,8 --assign balanced --reps 3 --out $O/rank_$n.jsonl > $O/rank_$n.log 2>&1 || { tail -5 $O/rank_$n.log; exit 1; }
  python3 -c "import sys,json; [print('$n', d['world'], d['max_ms'], d['mean_ms'], d['imbalance'], d.get('efficiency_vs_n1')) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_$n.jsonl
done
