#!/bin/bash
# A/B of library variants: GPU parity of the default build, then per variant a short bench and
# the per-pass kernel times (VARIANTS="default head ..." -> lib/exp/librtamd_<v>.so)
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
[ -n "$SKIP_PARITY" ] || timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
[ -n "$SKIP_PARITY" ] || tail -1 $O/parity.log
for v in ${VARIANTS:-default head}; do
  if [ $v = default ]; then L=""; else L=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_$v.so; fi
  RTAMD_LIB=$L timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --cpu-seconds 0 > $O/bench_$v.log 2>&1 || exit 1
  echo "$v: $(python3 -c "import json;d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_frame'],d['kernel']['avg_launch_ms'])")"
  [ -n "$SKIP_PASSES" ] && continue
  RTAMD_LIB=$L RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$v -o run -- python3 tools/quick_perf.py --frames 64 --per-launch 64 > $O/tr_$v.log 2>&1 || exit 1
  python3 tools/pass_profile.py $O/tr_$v/run_kernel_trace.csv | sed -n 4,6p
done
if [ -n "$SHPROF" ]; then
  RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_shprof.so timeout -k 10 200 python3 tools/quick_perf.py --frames 128 --per-launch 128 > $O/shprof.log 2>&1 || exit 1
  grep shade-prof $O/shprof.log | tail -1
fi
