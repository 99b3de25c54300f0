#!/bin/bash
# N = 8 rank shares on one GPU (tools/rank_sim.py) for frame-group counts / builds (development aid).
#   gpurun -- bash tools/rank_ab.sh <tag> "2 3 4"
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-rank}
O=gpurun_out/$TAG
mkdir -p $O
DEV=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
for G in ${2:-2 3 4}; do
  RTAMD_LIB=$DEV RT_GROUPS=$G RT_FAST_TRACE=${FAST:-1} timeout -k 10 600 python3 tools/rank_sim.py --worlds 1,8 --assign both --reps 2 \
    --out $O/groups$G.jsonl > $O/groups$G.log 2>&1 || { tail -5 $O/groups$G.log; exit 1; }
  echo "groups $G:"; cat $O/groups$G.jsonl | python3 -c "import sys,json; [print(' ', d['world'], d['assign'], d['max_ms'], d['mean_ms'], d['imbalance'], d['efficiency_vs_n1']) for d in map(json.loads, sys.stdin)]"
done
