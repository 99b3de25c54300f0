# SQ counters per kernel, one frame group (no overlap), 64 frames
export TMPDIR=/tmp
RT_GROUPS=1 QP="--frames 64 --per-launch 64 --count-frames 1" bash tools/pmc_sq.sh gpurun_out/sq6 || { echo pmc failed; tail gpurun_out/sq6/*.log; exit 1; }
python3 tools/pmc_report.py gpurun_out/sq6 > gpurun_out/sq6/report.txt
cat gpurun_out/sq6/report.txt
