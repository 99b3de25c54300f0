#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats (kernels co-run as in the bench).  Then PMC passes, one counter
# group per run (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950; SQ takes 8 slots,
# GRBM 2), each with its own --kernel-trace (counter collection serialises the dispatches, so
# these durations are standalone launches), never combined with --sys-trace / runtime / hip /
# memory-copy domains.
set -euo pipefail
OUT=${1:-gpurun_out/prof}
ARGS=${BENCH_ARGS:-"--steps 3 --warmup 1 --cpu-seconds 0 --single-frames 0"}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, rocprofv3 options...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 bench.py $ARGS > "$OUT/$name.log" 2>&1
  echo "profile pass $name done"
}
run trace --kernel-trace --stats
run pmc_fetch --kernel-trace --pmc FETCH_SIZE
run pmc_write --kernel-trace --pmc WRITE_SIZE
run pmc_sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run pmc_sq2 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT
run pmc_tcc --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum
echo profile-done
