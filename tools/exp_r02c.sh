#!/bin/bash
# GPU tests, single-frame sweep (finisher / static claims / tile order vs HEAD), bulk A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
X=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "head:RTAMD_LIB=$X/librtamd_head.so" "new:" "nofin:RT_FINISH_PASS=0" "sf0:RTAMD_LIB=$X/librtamd_sf0.so" "sf6:RTAMD_LIB=$X/librtamd_sf6.so" "p3:RT_FINISH_PASS=3" "p4:RT_FINISH_PASS=4"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --frames-per-step 64 --cpu-seconds 0 --single-frames 64 > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  echo "$n: $(python3 -c "import json;d=json.load(open('$O/b_$n.json'));print(d['value'],d['ms_per_frame'],d['ms_per_frame_single'],d['ms_single_frame_latency'])")"
done
timeout -k 10 500 python3 tools/ab_proc.py --rounds 3 --whole base=$X/librtamd_head.so new=default sf0=$X/librtamd_sf0.so > $O/ab_C3.log 2>&1 || { tail -20 $O/ab_C3.log; exit 1; }
tail -4 $O/ab_C3.log
