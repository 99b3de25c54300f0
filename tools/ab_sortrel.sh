export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
for v in base rel; do if [ $v = rel ]; then export RTAMD_LIB=$PWD/$L/librtamd_rel.so; else unset RTAMD_LIB; fi; for k in 1 2; do timeout -k 10 200 python3 tools/rank_sim.py --frames 1024 --reps 1 --worlds 8 2>/dev/null | grep world | sed "s/^/$v /"; done; done
unset RTAMD_LIB
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default rel=$L/librtamd_rel.so > gpurun_out/ab32.log 2>&1 || { echo ab failed; exit 1; }
tail -3 gpurun_out/ab32.log
