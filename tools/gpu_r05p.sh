#!/bin/bash
# round 5: per-segment claim counters in the bulk passes (parity on the variant, A/B, N=8 rank shares)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_x2.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/tests_x2.log 2>&1 || { echo "x2 tests failed"; tail -20 $O/tests_x2.log; exit 1; }
tail -1 $O/tests_x2.log
V=""
for n in base11 x1 x2 x4; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -5 $O/bulk.log
for n in base11 x2; do
  RTAMD_LIB=$E/librtamd_$n.so timeout -k 10 400 python3 tools/rank_sim.py --worlds 1,8 --assign balanced --reps 2 --out $O/rank_$n.jsonl > $O/rank_$n.log 2>&1 || { tail -5 $O/rank_$n.log; exit 1; }
  python3 -c "import sys,json; [print('$n', d['world'], d['max_ms'], d['mean_ms'], d['imbalance'], d.get('efficiency_vs_n1')) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_$n.jsonl
done
