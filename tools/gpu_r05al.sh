#!/bin/bash
# round 5: the bulk's smallest guided claim (32 / 128); the small passes' refill threshold (12 / 28)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05al; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 800 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 base27=$E/librtamd_base27.so gm32=$E/librtamd_gm32.so gm128=$E/librtamd_gm128.so > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -4 $O/bulk.log
timeout -k 10 500 python3 -u tools/ab_single.py --config C3 --rounds 3 base27=$E/librtamd_base27.so rs12=$E/librtamd_rs12.so rs28=$E/librtamd_rs28.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -4 $O/single.log
