#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/sp
for f in opengl-ray-tracing-framework_amd/lib/exp/librtamd_*.so; do
  n=$(basename $f .so)
  RTAMD_LIB=$PWD/$f RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sp/$n -o run -- python3 tools/quick_perf.py --frames 64 --per-launch 64 > gpurun_out/sp/$n.log 2>&1 || exit 1
  echo "== $n"; python3 tools/pass_profile.py gpurun_out/sp/$n/run_kernel_trace.csv | sed -n 4,6p
done
