#!/bin/bash
# round 5: which shade passes sort their paths by key (camera pass; every pass above 64 K paths)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aa; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base18 sp0 sall sp0all; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 $V > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -5 $O/bulk.log
