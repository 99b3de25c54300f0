#!/bin/bash
# SQ counters of one-frame render calls (development aid; run on the GPU box from the repo root):
# two PMC passes over tools/pass_counts.py (8 warm-up calls + 1), then tools/single_pmc.py.
set -euo pipefail
OUT=${1:-gpurun_out/spmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 120 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- python3 tools/pass_counts.py --order $PC_ARGS > "$OUT/$name.log" 2>&1
  echo "pass $name done"
}
PC_ARGS=${PC_ARGS:-}
run sq --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY
run sq2 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS
python3 tools/single_pmc.py "$OUT"
