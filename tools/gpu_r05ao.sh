#!/bin/bash
# round 5: one-frame shade paths per thread (small groups)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ao; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base30 ss1 ss2; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 700 python3 -u tools/ab_single.py --config C3 --rounds 4 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -4 $O/single.log
