set -e
cd /root/repo
mkdir -p gpurun_out/pipe5
RT_DEBUG=1 RT_AB_ORDER=1 RT_AB_PIPE=2 timeout -k 10 100 python3 tools/ab_single.py --one default --calls 8 2>&1 | grep -v "occupancy(lds" | head -20
timeout -k 10 600 python3 tools/ab_single.py --rounds 3 p2=default:RT_AB_ORDER=1,RT_AB_PIPE=2 \
  p2b2=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_PIPE_FINISH_BPC=2 \
  p2b3=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_PIPE_FINISH_BPC=3 > gpurun_out/pipe5/ab.log 2>&1
tail -4 gpurun_out/pipe5/ab.log
