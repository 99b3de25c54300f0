# pipelined one-frame calls: finisher occupancy / start pass A/B (development aid)
set -e
cd /root/repo
mkdir -p gpurun_out/pipe3
timeout -k 10 600 python3 tools/ab_single.py --rounds 2 p2=default:RT_AB_ORDER=1,RT_AB_PIPE=2 \
  bpc1=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_FINISH_BPC=1 \
  f3=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_FINISH_PASS=3 \
  f1=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_FINISH_PASS=1 \
  p3bpc1=default:RT_AB_ORDER=1,RT_AB_PIPE=3,RT_FINISH_BPC=1 > gpurun_out/pipe3/ab.log 2>&1
cat gpurun_out/pipe3/ab.log
