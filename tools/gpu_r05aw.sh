#!/bin/bash
# round 5: paths per thread of the small-group (one-frame) shade kernels, 3 / 2 / 1 (one-frame A/B)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aw; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds 4 ss3=$E/librtamd_ss3.so ss2=$E/librtamd_ss2.so ss1=$E/librtamd_ss1.so > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -5 $O/single.log
