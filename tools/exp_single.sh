#!/bin/bash
# single-frame latency (one frame per rt_render call, the reference's usage): pixel-split groups
# vs none, plus 4 groups, and the per-pass trace of the default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/single
mkdir -p $O
for cfg in "default:" "nosplit:RT_PIX_SPLIT=0" "g4:RT_GROUPS=4" "g3:RT_GROUPS=3"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --cpu-seconds 0 --single-frames 64 > $O/b_$n.json 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  echo "$n: $(python3 -c "import json;d=json.load(open('$O/b_$n.json'));print(d['value'],d['ms_per_frame'],d['ms_per_frame_single'],d['ms_single_frame_latency'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 tools/quick_perf.py --frames 16 --per-launch 1 > $O/tr.log 2>&1 || exit 1
python3 tools/pass_profile.py $O/tr/run_kernel_trace.csv | tail -8
