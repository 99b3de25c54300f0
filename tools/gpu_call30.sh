export TMPDIR=/tmp
for v in "base:" "c512:RT_POOL_CHUNK=512" "g3:RT_GROUPS=3" "g4:RT_GROUPS=4" "g1:RT_GROUPS=1"; do n=${v%%:*}; e=${v#*:}; env $e timeout -k 10 200 python3 tools/rank_sim.py --frames 1024 --reps 1 --worlds 8 2>/dev/null | grep world | sed "s/^/$n /"; done
