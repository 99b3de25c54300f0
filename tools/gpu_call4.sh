# SAH leaf weights for the rebuilt levels: triangles (default), 1 per leaf (-1), triangles + 4, + 16
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 0 -1 4 16; do RT_REBUILD_LEAFW=$w timeout -k 10 200 python3 tools/quick_perf.py --frames 64 --per-launch 64 --count-frames 8 2>&1 | grep -E "visits" | sed "s/^/w=$w /"; done
timeout -k 10 600 python3 tools/ab_proc.py --whole --rounds 3 t=default l1=default:RT_REBUILD_LEAFW=-1 t4=default:RT_REBUILD_LEAFW=4 t16=default:RT_REBUILD_LEAFW=16 > gpurun_out/ab4.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab4.log; exit 1; }
tail -5 gpurun_out/ab4.log
