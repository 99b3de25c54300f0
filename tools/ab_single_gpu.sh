#!/bin/bash
# One-frame-call A/B on the GPU (tools/ab_single.py variants: frames in flight, finisher settings,
# work order ...).  Development aid; the log lands in gpurun_out/single_<config>/ab.log.
#   gpurun -- bash tools/ab_single_gpu.sh C3 one=default:RT_AB_ORDER=1 two=default:RT_AB_ORDER=1,RT_AB_PIPE=2
set -e
cd /root/repo
export TMPDIR=/tmp
CFG=${1:-C3}; shift
O=gpurun_out/single_$CFG
mkdir -p $O
timeout -k 10 600 python3 tools/ab_single.py --config $CFG --rounds 2 "$@" > $O/ab.log 2>&1
tail -$(( $# + 1 )) $O/ab.log
