export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 1000 python3 tools/ab_proc.py --whole --rounds 3 base=default t128=$L/librtamd_t128.so t256=$L/librtamd_t256.so f2=$L/librtamd_f2.so f8=$L/librtamd_f8.so > gpurun_out/ab24.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab24.log; exit 1; }
tail -6 gpurun_out/ab24.log
