#!/bin/bash
# round 5: tail claims (exact idle-lane counts, lower refill threshold) and static shares
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 700 python3 -u tools/ab_single.py --config C3 --rounds 3 base=$E/librtamd_base6.so tx=$E/librtamd_tx.so \
  tx8=$E/librtamd_tx8.so tx1=$E/librtamd_tx1.so sf5=$E/librtamd_sf5.so sf6=$E/librtamd_sf6.so sf7=$E/librtamd_sf7.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -8 $O/single.log
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 base=$E/librtamd_base6.so \
  tx=$E/librtamd_tx.so tx8=$E/librtamd_tx8.so > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -4 $O/bulk.log
