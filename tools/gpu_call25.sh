export TMPDIR=/tmp
RT_GROUPS=1 QP="--frames 64 --per-launch 64 --count-frames 1" bash tools/pmc_sq.sh gpurun_out/sq25 || { echo pmc failed; tail gpurun_out/sq25/*.log; exit 1; }
python3 tools/pmc_report.py gpurun_out/sq25 > gpurun_out/sq25/report.txt
grep -E "^rtd|->" gpurun_out/sq25/report.txt
RT_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pp25/t -o run -- python3 tools/quick_perf.py --frames 320 --per-launch 160 > gpurun_out/pp25.log 2>&1 || { echo fail; exit 1; }
f=$(find gpurun_out/pp25/t -name '*kernel_trace.csv' | head -1)
python3 tools/pass_profile.py $f | tail -4
