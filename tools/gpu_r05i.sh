#!/bin/bash
# round 5: small-pass claim experiments (one-frame calls, then the bulk)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds 3 base=$E/librtamd_base5.so tc256=$E/librtamd_tc256.so \
  sf6=$E/librtamd_sf6.so sf8=$E/librtamd_sf8.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -6 $O/single.log
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 2 base=$E/librtamd_base5.so \
  tc256=$E/librtamd_tc256.so > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -3 $O/bulk.log
