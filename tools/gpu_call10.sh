export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default wpe5=$L/librtamd_wpe5.so wpe3=$L/librtamd_wpe3.so sub2=$L/librtamd_sub2.so sub8=$L/librtamd_sub8.so g3=default:RT_GROUPS=3 > gpurun_out/ab10.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab10.log; exit 1; }
tail -7 gpurun_out/ab10.log
