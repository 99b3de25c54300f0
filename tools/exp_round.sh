#!/bin/bash
# GPU parity (all -m gpu tests), the interactive loop at 1080p, then A/B variants
export TMPDIR=/tmp
O=gpurun_out/rnd
mkdir -p $O
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 300 python3 tools/interactive_demo.py --config C3 --frames 30 --out $O > $O/interactive.log 2>&1 || { tail -20 $O/interactive.log; exit 1; }
cat $O/interactive.log
SKIP_PARITY=1 VARIANTS="${VARIANTS:-default}" bash tools/exp_ab.sh
