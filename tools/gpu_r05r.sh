#!/bin/bash
# round 5: end-of-launch statistics flushes (sharded lines; none, measurement only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
RTAMD_LIB=$E/librtamd_shard.so timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_api.py tests/test_gpu_parity.py > $O/tests_shard.log 2>&1 || { echo "shard tests failed"; tail -20 $O/tests_shard.log; exit 1; }
tail -1 $O/tests_shard.log
V=""
for n in base12 shard nostat; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -4 $O/bulk.log
timeout -k 10 400 python3 -u tools/ab_single.py --config C3 --rounds 3 base12=$E/librtamd_base12.so shard=$E/librtamd_shard.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -3 $O/single.log
