#!/bin/bash
# rocprofv3 kernel trace + PMC passes (tools/profile_gpu.sh) of C4 and C5 at 256-frame steps, their
# summaries into profiles/ (pmc_C4.json, pmc_C5.json), then each configuration's bench line, which
# reads them (roofline with traffic and VALU figures, cpu_baseline).
#   gpurun -- bash tools/profile_configs.sh <round tag, e.g. r05>
set -o pipefail
export TMPDIR=/tmp
R=${1:-r05}
mkdir -p gpurun_out/profiles
for c in ${CONFIGS:-C4 C5}; do
  case $c in C5) W=3840; H=2160; S=2139095040 ;; *) W=1920; H=1080; S=534773760 ;; esac
  BENCH_ARGS="--config $c --frames-per-step 256 --steps 3 --warmup 1 --cpu-seconds 0 --single-frames 0" \
    bash tools/profile_gpu.sh gpurun_out/prof_$c || { echo "profile $c failed"; exit 1; }
  python3 tools/summarize_profile.py gpurun_out/prof_$c ${R}_$c \
    "{\"config\": \"$c\", \"width\": $W, \"height\": $H, \"frames_per_step\": 256, \"path_slots_per_rank\": $S, \"probe_trace_launches\": 9, \"command\": \"BENCH_ARGS='--config $c --frames-per-step 256 --steps 3 --warmup 1 --cpu-seconds 0 --single-frames 0' bash tools/profile_gpu.sh\"}" > gpurun_out/summary_$c.log || { echo "summary $c failed"; exit 1; }
  cp profiles/${R}_${c}_* profiles/pmc_$c.json gpurun_out/profiles/
  timeout -k 10 600 python3 bench.py --config $c --frames-per-step 256 --steps 3 --warmup 1 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { echo "bench $c failed"; tail gpurun_out/bench_$c.err; exit 1; }
  cp gpurun_out/bench_$c.json gpurun_out/profiles/${R}_bench_$c.json
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$c.json'));r=d['roofline'];print('$c', d['value'], d['ms_per_frame'], d.get('ms_single_frame_latency'), r['bound'], r['frac'], r.get('traffic'), d['cpu_baseline']['value'])"
done
