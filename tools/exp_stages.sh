#!/bin/bash
# staged camera-path generation: parity at RT_STAGES=1 and 3, then process-level A/B
export TMPDIR=/tmp
O=gpurun_out/stg
mkdir -p $O
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $O/parity1.log 2>&1 || { tail -30 $O/parity1.log; exit 1; }
tail -1 $O/parity1.log
RT_STAGES=3 timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $O/parity3.log 2>&1 || { tail -30 $O/parity3.log; exit 1; }
tail -1 $O/parity3.log
timeout -k 10 1300 python3 tools/ab_proc.py --rounds 2 s1=default s2=default:RT_STAGES=2 s4=default:RT_STAGES=4 s8=default:RT_STAGES=8 s16=default:RT_STAGES=16 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v round $O/ab.log | grep -v amdgpu.ids
