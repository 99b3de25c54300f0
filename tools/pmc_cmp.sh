#!/bin/bash
# Per-variant counters of one frame group (RT_GROUPS=1: no kernel overlap), quick_perf workload:
# kernel trace (durations), SQ issue counters, L2 hits.  VARIANTS="default name ..."
# (name -> lib/exp/librtamd_<name>.so); WRITES=1 adds a WRITE_SIZE pass (alone: it takes 2 of the 4 TCC counters, FETCH_SIZE 3).  Summary per kernel: tools/pmc_cmp.py
set -o pipefail
export TMPDIR=/tmp RT_GROUPS=1
O=gpurun_out/pmc_cmp
mkdir -p $O
QP=${QP:---frames 64 --per-launch 64}
for v in ${VARIANTS:-default}; do
  if [ $v = default ]; then L=""; else L=$PWD/opengl-ray-tracing-framework_amd/lib/exp/librtamd_$v.so; fi
  export RTAMD_LIB=$L
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$v/t -o run -- python3 tools/quick_perf.py $QP > $O/$v.t.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU --output-format csv -d $O/$v/a -o run -- python3 tools/quick_perf.py $QP > $O/$v.a.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $O/$v/b -o run -- python3 tools/quick_perf.py $QP > $O/$v.b.log 2>&1 || exit 1
  if [ -n "$WRITES" ]; then
    timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/$v/c -o run -- python3 tools/quick_perf.py $QP > $O/$v.c.log 2>&1 || exit 1
  fi
  echo "$v done"
done
python3 tools/pmc_cmp.py $O ${VARIANTS:-default}
