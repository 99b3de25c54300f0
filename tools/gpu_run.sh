#!/bin/bash
# The one GPU-box runner (development aid): a tag, then steps run in order, each under its own time
# limit, stopping at the first failure.  Logs land in gpurun_out/<tag>/.
#
#   gpurun -- bash tools/gpu_run.sh <tag> <step> [<step> ...]
#
# Steps (a variant is a library lib/exp/librtamd_<name>.so, built on the CPU side with
# `make -C opengl-ray-tracing-framework_amd variant_rel NAME=<name> HIPEXTRA=...` or
# `NAME=<name> tools/build_head_variant.sh`; "default" is lib/librtamd.so; name=lib:VAR=v,... sets
# environment for that variant, dev-library knobs need a `variant` build):
#   tests[=<pytest args>]   GPU suite (-m gpu), or the given files / -k expression
#   smoke                   __graft_entry__.smoke()
#   ab=<v>,<v>,...          C3 whole 1024-frame steps, process per measurement (tools/ab_proc.py)
#   ab4=<v>,<v>,...         C4 256-frame calls
#   single=<v>,<v>,...      C3 one-frame calls (tools/ab_single.py)
#   rank=<spec> ...         N = 8 rank shares on one GPU (tools/rank_sim.py); spec: VAR=v,VAR=v or "-"
#   passes=<cfg>:<frames>[:VAR=v;VAR=v][:count]  per-pass times (or visit counts) of one frame group
#                           (dev library)
#   bench[=<bench.py args>] the driver's bench command (default args: --gpus 1 --steps 20 --warmup 5)
#   configs                 bench lines of C2, C4, C5 (256-frame steps)
#   evidence[=<tag>]        round evidence: tests, rocprofv3 trace + PMC summary, bench, interactive
#                           (tools/round_gpu.sh)
#   profile_configs=<round> C4 / C5 rocprofv3 trace + PMC summaries and bench lines
#                           (tools/profile_configs.sh), then the C2 bench line
set -o pipefail
export TMPDIR=/tmp
TAG=${1:?usage: gpu_run.sh <tag> <step> ...}; shift
O=gpurun_out/$TAG; mkdir -p $O
E=$PWD/opengl-ray-tracing-framework_amd/lib/exp
ROUNDS=${ROUNDS:-3}

variants() {  # "a,b:X=1" -> "a=<lib> b=<lib>:X=1"
  local out="" v name rest lib envs
  IFS=',' read -ra vs <<< "$1"
  for v in "${vs[@]}"; do
    name=${v%%:*}; rest=""; [ "$v" != "$name" ] && rest=":${v#*:}"
    lib=default; [ "$name" != default ] && lib=$E/librtamd_$name.so
    out="$out $name=$lib${rest//;/,}"
  done
  echo $out
}
fail() { echo "step $1 failed (rc $2)"; tail -30 "$3"; exit 1; }

n=0
for step in "$@"; do
  n=$((n + 1)); key=${step%%=*}; arg=""; [ "$step" != "$key" ] && arg=${step#*=}
  L=$O/$n.$key.log
  case $key in
    tests)
      timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${arg:-tests} > $L 2>&1 || fail $step $? $L
      tail -1 $L ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $L 2>&1 || fail $step $? $L
      tail -1 $L ;;
    ab)
      timeout -k 10 1000 python3 -u tools/ab_proc.py --frames 1024 --whole --reps 2 --rounds $ROUNDS $(variants $arg) > $L 2>&1 || fail $step $? $L
      grep -A20 "^median" $L ;;
    ab4)
      timeout -k 10 600 python3 -u tools/ab_proc.py --config C4 --frames 256 --reps 2 --rounds 2 $(variants $arg) > $L 2>&1 || fail $step $? $L
      grep -A20 "^median" $L ;;
    single)
      timeout -k 10 600 python3 -u tools/ab_single.py --config C3 --rounds $ROUNDS $(variants $arg) > $L 2>&1 || fail $step $? $L
      tail -6 $L ;;
    rank)
      name=$(echo "${arg:--}" | tr ',=' '_-')
      envs=(); [ "${arg:--}" != "-" ] && IFS=',' read -ra envs <<< "$arg"
      env "${envs[@]}" RTAMD_LIB=$PWD/opengl-ray-tracing-framework_amd/lib/librtamd_dev.so timeout -k 10 600 \
        python3 tools/rank_sim.py --worlds ${WORLDS:-1,8} --assign ${ASSIGN:-balanced} --tile ${TILE:-16} --reps 2 --out $O/rank_$name.jsonl > $L 2>&1 || fail $step $? $L
      python3 -c "import sys,json; [print(' ', d['world'], d['assign'], d['max_ms'], d['mean_ms'], d['imbalance'], d['efficiency_vs_n1']) for d in map(json.loads, open(sys.argv[1]))]" $O/rank_$name.jsonl ;;
    passes)  # passes=<config>:<frames>[:VAR=v;VAR=v][:count]
      IFS=':' read -r cfg fr penv pcount <<< "$arg"
      envs=(); [ -n "$penv" ] && IFS=';' read -ra envs <<< "$penv"
      env "${envs[@]}" RT_DEBUG_PASSES=1 RT_GROUPS=1 timeout -k 10 300 \
        python3 -u tools/pass_counts.py --config $cfg --frames $fr --max-paths $((fr * 1920 * 1080)) ${pcount:+--count} > $L 2>&1 || fail $step $? $L
      grep -a "\] group\|pass" $L | head -30 ;;
    bench)
      timeout -k 10 600 python3 bench.py ${arg:---gpus 1 --steps 20 --warmup 5} > $O/bench.json 2> $L || fail $step $? $L
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['value'], d['ms_per_frame'], d.get('ms_single_frame_latency'), d.get('ms_per_frame_single'), d['roofline']['frac'])" $O/bench.json ;;
    configs)
      for c in C2 C4 C5; do
        timeout -k 10 300 python3 bench.py --config $c --frames-per-step 256 --steps 3 --warmup 1 --cpu-seconds 0 > $O/bench_$c.json 2> $L || fail $step $? $L
        python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('$c', d['value'], d['ms_per_frame'], d.get('ms_single_frame_latency'), d['rays_per_sample'], d['own_traversal_per_ray'])" $O/bench_$c.json
      done ;;
    evidence)
      TAG=${arg:-r06_C3} bash tools/round_gpu.sh > $L 2>&1 || fail $step $? $L
      tail -20 $L ;;
    profile_configs)
      bash tools/profile_configs.sh ${arg:-r06} > $L 2>&1 || fail $step $? $L
      grep -E "^C[45] " $L
      timeout -k 10 300 python3 bench.py --config C2 --frames-per-step 256 --steps 3 --warmup 1 > gpurun_out/profiles/${arg:-r06}_bench_C2.json 2>> $L || fail $step $? $L
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('C2', d['value'], d['ms_per_frame'], d.get('ms_single_frame_latency'), d.get('ms_per_frame_single'))" gpurun_out/profiles/${arg:-r06}_bench_C2.json ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
