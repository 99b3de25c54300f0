#!/bin/bash
# wf_finish: GPU parity tests (small calls take the finisher by default), then single-frame
# latency per finisher pass / occupancy variant (development aid)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/finish
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
X=$PWD/opengl-ray-tracing-framework_amd/lib/exp
for cfg in ${CFGS:-"off:RT_FINISH_PASS=0" "p1:RT_FINISH_PASS=1" "p2:RT_FINISH_PASS=2" "p3:RT_FINISH_PASS=3" "p4:RT_FINISH_PASS=4" "fw2p2:RTAMD_LIB=$X/librtamd_fw2.so" "fw3p2:RTAMD_LIB=$X/librtamd_fw3.so"}; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --frames-per-step 64 --cpu-seconds 0 --single-frames 64 > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  echo "$n: $(python3 -c "import json;d=json.load(open('$O/b_$n.json'));print(d['value'],d['ms_per_frame'],d['ms_per_frame_single'],d['ms_single_frame_latency'])")"
done
