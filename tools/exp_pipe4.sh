# pipelined one-frame calls: finisher start pass with the half-occupancy finisher (development aid)
set -e
cd /root/repo
mkdir -p gpurun_out/pipe4
timeout -k 10 600 python3 tools/ab_single.py --rounds 2 p2=default:RT_AB_ORDER=1,RT_AB_PIPE=2 \
  p2f3=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_PIPE_FINISH_PASS=3 \
  p2f4=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_PIPE_FINISH_PASS=4 \
  p3f3=default:RT_AB_ORDER=1,RT_AB_PIPE=3,RT_PIPE_FINISH_PASS=3 \
  p2b2=default:RT_AB_ORDER=1,RT_AB_PIPE=2,RT_PIPE_FINISH_BPC=2 > gpurun_out/pipe4/ab.log 2>&1
cat gpurun_out/pipe4/ab.log
