#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O
timeout -k 10 1100 python3 tools/ab_single.py --rounds 2 p3g2=default p2g2=default:RT_FINISH_PASS=2 p1g2=default:RT_FINISH_PASS=1 p3g4=default:RT_GROUPS=4 p2g4=default:RT_FINISH_PASS=2,RT_GROUPS=4 p1g4=default:RT_FINISH_PASS=1,RT_GROUPS=4 p2g3=default:RT_FINISH_PASS=2,RT_GROUPS=3 p2g1=default:RT_FINISH_PASS=2,RT_GROUPS=1 > $O/ab_single.log 2>&1 || { tail -20 $O/ab_single.log; exit 1; }
tail -9 $O/ab_single.log
