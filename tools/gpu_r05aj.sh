#!/bin/bash
# round 5: small passes prefetch one dword of the iteration's node / the next triangle (one-frame A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aj; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
V=""
for n in base24 npf tpf ntpf; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds 3 $V > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -5 $O/single.log
