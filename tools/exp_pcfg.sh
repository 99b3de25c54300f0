# one-frame calls on the other configurations, one and two in flight (development aid)
set -e
cd /root/repo
mkdir -p gpurun_out/pcfg
for c in C2 C4 C5; do
  timeout -k 10 400 python3 tools/ab_single.py --config $c --rounds 1 --calls 24 one=default:RT_AB_ORDER=1 two=default:RT_AB_ORDER=1,RT_AB_PIPE=2 > gpurun_out/pcfg/$c.log 2>&1
  echo "== $c"; tail -2 gpurun_out/pcfg/$c.log
done
