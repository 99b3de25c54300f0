export TMPDIR=/tmp
mkdir -p gpurun_out/exp
for g in 768 256 64; do
 for sz in "64 64" "480 270" "1920 1080"; do
  set -- $sz
  RT_TRACE_GRID=$g timeout -k 10 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/exp/g${g}_$1 -o run -- python3 tools/quick_perf.py --frames 4 --per-launch 4 --max-bounce 0 --width $1 --height $2 > gpurun_out/exp/g${g}_$1.log 2>&1 || exit 1
 done
done
echo ok
