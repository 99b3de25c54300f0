#!/bin/bash
# round 5: compiler scheduling strategies
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ai; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base23 ilp mclause trk bias0; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -6 $O/bulk.log
