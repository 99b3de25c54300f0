# pipelined batches: one rank's share at N = 8 / 4 and the whole frame at N = 1 (development aid)
set -e
cd /root/repo
mkdir -p gpurun_out/pbatch
for args in "--worlds 8 --assign balanced" "--worlds 8 --assign balanced --pipeline 2" \
            "--worlds 4 --assign balanced" "--worlds 4 --assign balanced --pipeline 2" \
            "--worlds 1 --assign modulo" "--worlds 1 --assign modulo --pipeline 2 --calls 4"; do
  echo "== $args"
  timeout -k 10 240 python3 tools/rank_sim.py --reps 2 $args 2>&1 | grep '^{' | python3 -c "import sys,json;[print(json.dumps({k:d[k] for k in ('world','pipeline','calls','max_ms','mean_ms','imbalance','mrays_per_s_job')})) for d in map(json.loads,sys.stdin)]"
done
