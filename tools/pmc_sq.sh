#!/bin/bash
# SQ stall / utilisation counters per kernel for the quick_perf workload.
export TMPDIR=/tmp
OUT=${1:-gpurun_out/sq}
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/a -o run -- python3 tools/quick_perf.py ${QP:---frames 4 --per-launch 4} > $OUT/a.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA --output-format csv -d $OUT/b -o run -- python3 tools/quick_perf.py ${QP:---frames 4 --per-launch 4} > $OUT/b.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $OUT/c -o run -- python3 tools/quick_perf.py ${QP:---frames 4 --per-launch 4} > $OUT/c.log 2>&1 || exit 1
echo ok
