export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 split=default old=$L/librtamd_old.so w5=$L/librtamd_w5.so > gpurun_out/ab14.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab14.log; exit 1; }
tail -4 gpurun_out/ab14.log
