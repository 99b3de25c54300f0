#!/bin/bash
# round 5: refill queue-entry prefetch; a second triangle test in the node half (bulk and one-frame calls)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base8 rpf tri2 tri2rpf; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -5 $O/bulk.log
V=""
for n in base8 rpf tri2 tri2b; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds 3 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -5 $O/single.log
