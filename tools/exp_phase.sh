#!/bin/bash
# wf_shade phase breakdown (RT_SHADE_PROF variant) + shade lane utilisation counters
export TMPDIR=/tmp
mkdir -p gpurun_out/ph
L=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_shprof.so
RTAMD_LIB=$L timeout -k 10 200 python3 tools/quick_perf.py --frames 128 --per-launch 128 > gpurun_out/ph/prof.log 2>&1 || exit 1
grep -E "shade-prof|Mrays" gpurun_out/ph/prof.log | tail -3
timeout -k 10 300 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VALU --output-format csv -d gpurun_out/ph/pmc -o run -- python3 tools/quick_perf.py --frames 64 --per-launch 64 > gpurun_out/ph/pmc.log 2>&1 || exit 1
python3 tools/pmc_report.py gpurun_out/ph/pmc
for s in 160 320; do
  RT_MAX_SLOTS=$((s<<20)) timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --cpu-seconds 0 > gpurun_out/ph/bench_$s.log 2>&1 || exit 1
  echo "slots ${s}M: $(python3 -c "import json;d=json.loads(open('gpurun_out/ph/bench_$s.log').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_frame'])")"
done
