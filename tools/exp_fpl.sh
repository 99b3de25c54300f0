#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/fpl
for f in 16 32 64; do
  RT_MAX_SLOTS=140000000 timeout -k 10 300 python3 tools/quick_perf.py --frames $((f*3)) --per-launch $f > gpurun_out/fpl/f$f.log 2>&1 || exit 1
  echo "frames/launch $f: $(grep ms/frame gpurun_out/fpl/f$f.log)"
done
