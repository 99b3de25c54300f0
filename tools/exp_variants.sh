#!/bin/bash
# time every lib/exp/librtamd_*.so variant on C3 (development aid); first variant also parity-checked
export TMPDIR=/tmp
mkdir -p gpurun_out/var
for f in opengl-ray-tracing-framework_amd/lib/exp/librtamd_*.so; do
  n=$(basename $f .so)
  RTAMD_LIB=$PWD/$f timeout -k 10 200 python3 tools/quick_perf.py --frames 32 --per-launch 16 > gpurun_out/var/$n.log 2>&1 || { echo "$n failed"; exit 1; }
  echo "$n: $(grep ms/frame gpurun_out/var/$n.log)"
done
