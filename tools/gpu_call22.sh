export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 1000 python3 tools/ab_proc.py --whole --rounds 3 sm64=$L/librtamd_sm64.so sm32=$L/librtamd_sm32.so sm128=$L/librtamd_sm128.so sm256=$L/librtamd_sm256.so sm64l10=$L/librtamd_sm64.so:RT_LDS_STACK=10 > gpurun_out/ab22.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab22.log; exit 1; }
tail -6 gpurun_out/ab22.log
