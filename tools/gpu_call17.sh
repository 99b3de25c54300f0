export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default nosort=$L/librtamd_nosort.so keymat=$L/librtamd_keymat.so camdual=default:RT_TRACE_MODE0=3 c256=default:RT_POOL_CHUNK=256 c1024=default:RT_POOL_CHUNK=1024 > gpurun_out/ab17.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab17.log; exit 1; }
tail -7 gpurun_out/ab17.log
