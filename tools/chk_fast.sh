#!/bin/bash
# RT_CHECK build of the fast traversal on the bench workload at a small size (development aid).
cd /root/repo && export TMPDIR=/tmp && mkdir -p gpurun_out/chk
RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_fastchk.so AMD_SERIALIZE_KERNEL=3 timeout -k 10 240 \
  python -u bench.py --steps 1 --warmup 1 --frames-per-step 4 --width 256 --height 160 --cpu-seconds 0 --single-frames 0 \
  --frame-sha --gpus 1 > /tmp/b.log 2>&1
echo rc=$?
grep -a "rt check" /tmp/b.log | sed 's/[0-9]\{4,\}/N/g' | sort | uniq -c | sort -rn | head -30
grep -a "rt check" /tmp/b.log | head -20 > gpurun_out/chk/first.log
grep -av "rt check" /tmp/b.log | tail -c 3000
