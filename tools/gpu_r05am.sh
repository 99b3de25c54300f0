#!/bin/bash
# round 5: the small passes' refill threshold 4 / 6 / 8 vs 20 (one-frame A/B, 4 rounds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05am; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base28 rs4 rs6 rs8; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 700 python3 -u tools/ab_single.py --config C3 --rounds 4 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -5 $O/single.log
