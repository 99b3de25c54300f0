#!/bin/bash
# round 5: small-pass trace instantiations at other occupancies, with the finisher's prefetching step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base7 w4 spf4 spf5 spf6 spf6np; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 800 python3 -u tools/ab_single.py --config C3 --rounds 3 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -7 $O/single.log
