#!/bin/bash
# round 5: N=8 rank shares, segment claims vs one counter, interleaved (2 rounds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
for r in 1 2; do
for n in base11 x2 x4 x1; do
  RTAMD_LIB=$E/librtamd_$n.so timeout -k 10 400 python3 tools/rank_sim.py --worlds 8 --assign balanced --reps 3 --out $O/rank_${n}_$r.jsonl > $O/rank_${n}_$r.log 2>&1 || { tail -5 $O/rank_${n}_$r.log; exit 1; }
  python3 -c "import sys,json; [print('$n', d['world'], d['max_ms'], d['mean_ms'], d['imbalance']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_${n}_$r.jsonl
done
done
