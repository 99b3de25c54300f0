#!/bin/bash
# round 5: one-frame finisher knobs on the current build (shade batch, priority thresholds; finish pass, blocks per CU via the dev library)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ae; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
D=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
V=""
for n in base21 fsm8 fsm32 fp32 fp8; do V="$V $n=$E/librtamd_$n.so"; done
timeout -k 10 700 python3 -u tools/ab_single.py --config C3 --rounds 3 $V dev=$D dfp1=$D:RT_FINISH_PASS=1 dfp3=$D:RT_FINISH_PASS=3 dbpc2=$D:RT_FINISH_BPC=2 > $O/single.log 2>&1 || { tail -20 $O/single.log; exit 1; }
tail -10 $O/single.log
