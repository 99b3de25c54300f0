export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default w7=$L/librtamd_w7.so w6=$L/librtamd_w6.so > gpurun_out/ab12.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab12.log; exit 1; }
tail -4 gpurun_out/ab12.log
