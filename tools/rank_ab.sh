#!/bin/bash
# N = 1 / 8 rank-share A/B of release-like variants (lib/exp/librtamd_<name>.so), interleaved rounds:
#   gpurun -- bash tools/rank_ab.sh <tag> <name> <name> ...
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_$v.so timeout -k 10 300 python3 tools/rank_sim.py \
      --worlds 1,8 --assign balanced --tile 16 --reps 2 --out $O/${v}_$r.jsonl > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
    python3 -c "import sys,json; L=[json.loads(x) for x in open(sys.argv[1])]; print(sys.argv[2], ' '.join('%d:%.1f/%.4f' % (d['world'], d['max_ms'], d['efficiency_vs_n1']) for d in L))" $O/${v}_$r.jsonl $v
  done
done
