export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 1000 python3 tools/ab_proc.py --whole --rounds 3 base=default sm4=$L/librtamd_sm4.so sm64=$L/librtamd_sm64.so lds10=default:RT_LDS_STACK=10 lds7=default:RT_LDS_STACK=7 > gpurun_out/ab21.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab21.log; exit 1; }
tail -6 gpurun_out/ab21.log
