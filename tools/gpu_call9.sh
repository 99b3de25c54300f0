export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default rf8=$L/librtamd_rf8.so rf24=$L/librtamd_rf24.so rf32=$L/librtamd_rf32.so > gpurun_out/ab9.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab9.log; exit 1; }
tail -5 gpurun_out/ab9.log
