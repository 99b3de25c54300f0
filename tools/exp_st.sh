set -e
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/st
RT_AB_ORDER=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/st/prof -o run -- python3 tools/ab_single.py --one default --calls 24 > gpurun_out/st/ab.log 2>&1
f=$(find gpurun_out/st/prof -name '*kernel_trace.csv' | head -1)
python3 tools/single_timeline.py "$f" --calls 3 > gpurun_out/st/timeline.txt
cat gpurun_out/st/ab.log | tail -2
head -80 gpurun_out/st/timeline.txt
