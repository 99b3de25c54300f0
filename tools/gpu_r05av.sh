#!/bin/bash
# round 5: N=1 / N=8 rank shares with the frame groups staggered (group 1 starts after group 0's
# k-th launch; dev library, RT_GROUP_STAGGER)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05av; mkdir -p $O
DEV=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
for k in 0 1 2 3; do
  RT_GROUP_STAGGER=$k RTAMD_LIB=$DEV timeout -k 10 400 python3 tools/rank_sim.py --worlds 1,8 --assign balanced --reps 2 --tile 16 --out $O/stag$k.jsonl > $O/stag$k.log 2>&1 || { tail -5 $O/stag$k.log; exit 1; }
  python3 -c "import sys,json; [print('stagger $k', d['world'], d['max_ms'], d['mean_ms'], d['imbalance'], d.get('efficiency_vs_n1')) for d in map(json.loads, open(sys.argv[1]))]" $O/stag$k.jsonl
done
