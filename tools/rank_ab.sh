#!/bin/bash
# N = 8 rank shares on one GPU (tools/rank_sim.py) for development settings of the dev library
# (development aid).  Each spec is a comma-separated list of VAR=value (or "-" for none):
#   gpurun -- bash tools/rank_ab.sh <tag> "RT_GROUPS=2 RT_GROUPS=3 RT_FINISH_PASS=5,RT_FINISH_SLOTS=4000000000"
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
TAG=${1:-rank}
O=gpurun_out/$TAG
mkdir -p $O
DEV=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
WORLDS=${WORLDS:-1,8}
for spec in ${2:--}; do
  name=$(echo "$spec" | tr ',=' '_-')
  envs=()
  [ "$spec" != "-" ] && IFS=',' read -ra envs <<< "$spec"
  env "${envs[@]}" RTAMD_LIB=$DEV timeout -k 10 600 python3 tools/rank_sim.py --worlds $WORLDS --assign ${ASSIGN:-balanced} \
    --reps 2 --out $O/$name.jsonl > $O/$name.log 2>&1 || { tail -5 $O/$name.log; exit 1; }
  echo "$spec:"; python3 -c "import sys,json; [print(' ', d['world'], d['assign'], d['max_ms'], d['mean_ms'], d['imbalance'], d['efficiency_vs_n1']) for d in map(json.loads, open(sys.argv[1]))]" $O/$name.jsonl
done
