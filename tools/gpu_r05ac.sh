#!/bin/bash
# round 5: frame groups per launch (dev library knob RT_GROUPS) on the current build, bulk and N=8 shares
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ac; mkdir -p $O
D=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so
timeout -k 10 900 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds 3 g2=$D g3=$D:RT_GROUPS=3 g4=$D:RT_GROUPS=4 g1=$D:RT_GROUPS=1 > $O/bulk.log 2>&1 || { tail -20 $O/bulk.log; exit 1; }
tail -5 $O/bulk.log
WORLDS=1,8 bash tools/rank_ab.sh r05ac_rank "- RT_GROUPS=3 RT_GROUPS=4"
