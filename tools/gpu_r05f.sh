#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds 3 base=$E/librtamd_r05base.so:RT_AB_ORDER=1 climit=$E/librtamd_r05climit.so:RT_AB_ORDER=1 > $O/ab_single.log 2>&1 || { tail -20 $O/ab_single.log; exit 1; }
tail -3 $O/ab_single.log
