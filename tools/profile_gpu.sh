#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root).
# Pass 1: kernel trace + stats.  Passes 2-3: PMC counters, one block per pass (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass on gfx950), kernel trace only alongside.
set -euo pipefail
OUT=${1:-gpurun_out/prof}
ARGS=${BENCH_ARGS:-"--steps 5 --warmup 1 --cpu-seconds 0"}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py $ARGS > "$OUT/pmc_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py $ARGS > "$OUT/pmc_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py $ARGS > "$OUT/pmc_sq.log" 2>&1
echo profile-done
