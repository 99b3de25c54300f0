#!/bin/bash
# round 5: guided claim sizes, second round (divisor, first chunk, tail chunk); one-frame check
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base9 g2 g3 g2c2k g1c2k g2tc128; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -7 $O/bulk.log
timeout -k 10 400 python3 -u tools/ab_single.py --config C3 --rounds 3 base9=$E/librtamd_base9.so g2=$E/librtamd_g2.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -3 $O/single.log
