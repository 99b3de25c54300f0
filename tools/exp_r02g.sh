#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
B=4294967296
timeout -k 10 900 python3 tools/ab_proc.py --rounds 3 --whole base=default f4=default:RT_FINISH_SLOTS=$B,RT_FINISH_PASS=4 f5=default:RT_FINISH_SLOTS=$B,RT_FINISH_PASS=5 f6=default:RT_FINISH_SLOTS=$B,RT_FINISH_PASS=6 f7=default:RT_FINISH_SLOTS=$B,RT_FINISH_PASS=7 > $O/ab_C3.log 2>&1 || { tail -20 $O/ab_C3.log; exit 1; }
tail -6 $O/ab_C3.log
