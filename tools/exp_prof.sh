#!/bin/bash
# kernel trace (per pass) + SQ counters for the default trace configuration (development aid)
export TMPDIR=/tmp
OUT=gpurun_out/prof2
mkdir -p $OUT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/quick_perf.py --frames 8 --per-launch 4 > $OUT/kt.log 2>&1 || exit 1
bash tools/pmc_sq.sh $OUT/sq || exit 1
echo ok
