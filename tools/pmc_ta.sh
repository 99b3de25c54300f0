#!/bin/bash
# TA / TD / TCP busy counters (is the vector-memory address path the limiter?)
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ta}
mkdir -p $OUT
rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TA_BUSY_max TD_BUSY_avr --output-format csv -d $OUT/a -o run -- python3 tools/quick_perf.py --frames 4 --per-launch 4 > $OUT/a.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc TCP_TCR_TCP_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum --output-format csv -d $OUT/b -o run -- python3 tools/quick_perf.py --frames 4 --per-launch 4 > $OUT/b.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_GATE_EN1_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum --output-format csv -d $OUT/c -o run -- python3 tools/quick_perf.py --frames 4 --per-launch 4 > $OUT/c.log 2>&1 || exit 1
echo ok
