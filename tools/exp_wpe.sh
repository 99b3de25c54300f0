#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/wpe
for f in opengl-ray-tracing-framework_amd/lib/exp/librtamd_*.so; do
  n=$(basename $f .so)
  for k in 8 12; do
    RTAMD_LIB=$PWD/$f RT_LDS_STACK=$k RT_DEBUG=1 timeout -k 10 300 python3 tools/quick_perf.py --frames 128 --per-launch 64 > gpurun_out/wpe/${n}_k$k.log 2>&1 || exit 1
    echo "$n lds $k: $(grep ms/frame gpurun_out/wpe/${n}_k$k.log | cut -c1-80) $(grep 'trace: lds' gpurun_out/wpe/${n}_k$k.log | sed 's/.*using/using/')"
  done
done
