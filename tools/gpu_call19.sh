export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 1000 python3 tools/ab_proc.py --whole --rounds 3 base=default rf16=$L/librtamd_rf16.so rf32=$L/librtamd_rf32.so sub4=$L/librtamd_sub4.so sub1=$L/librtamd_sub1.so g3=default:RT_GROUPS=3 > gpurun_out/ab19.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab19.log; exit 1; }
tail -7 gpurun_out/ab19.log
