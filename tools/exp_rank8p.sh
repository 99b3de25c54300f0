# N = 8 rank shares with steps in flight: tile maps and tile sizes (development aid)
set -e
cd /root/repo
for args in "--assign balanced --pipeline 2 --reps 3" "--assign modulo --pipeline 2 --reps 3" "--assign balanced --pipeline 2 --reps 3 --tile 16" "--assign balanced --reps 3"; do
  echo "== $args"
  timeout -k 10 300 python3 tools/rank_sim.py --worlds 8 $args 2>&1 | grep '^{' | python3 -c "import sys,json;[print(json.dumps({k:d[k] for k in ('world','assign','pipeline','max_ms','mean_ms','imbalance','rank_ms')})) for d in map(json.loads,sys.stdin)]"
done
