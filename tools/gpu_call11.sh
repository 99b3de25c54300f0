export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default sub1=$L/librtamd_sub1.so sub2=$L/librtamd_sub2.so sub2m=$L/librtamd_sub2m.so sub2g3=$L/librtamd_sub2.so:RT_GROUPS=3 > gpurun_out/ab11.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab11.log; exit 1; }
tail -6 gpurun_out/ab11.log
