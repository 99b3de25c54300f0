# rolling chunk pipeline: parity, then A/B of the stagger pass vs the batch-barrier build
export TMPDIR=/tmp
L=opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest15.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/pytest15.log; exit 1; }
tail -1 gpurun_out/pytest15.log
timeout -k 10 900 python3 tools/ab_proc.py --whole --frames 1024 --reps 1 --rounds 2 old=$L/librtamd_old.so s2=default s1=default:RT_STAGGER=1 s3=default:RT_STAGGER=3 s4=default:RT_STAGGER=4 sn=default:RT_STAGGER=-1 > gpurun_out/ab15.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab15.log; exit 1; }
tail -7 gpurun_out/ab15.log
