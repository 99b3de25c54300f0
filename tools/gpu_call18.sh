export TMPDIR=/tmp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 c1024=default:RT_POOL_CHUNK=1024 c2048=default:RT_POOL_CHUNK=2048 c4096=default:RT_POOL_CHUNK=4096 c1024d=default:RT_POOL_CHUNK=1024,RT_TRACE_MODE0=3 c2048d=default:RT_POOL_CHUNK=2048,RT_TRACE_MODE0=3 > gpurun_out/ab18.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab18.log; exit 1; }
tail -6 gpurun_out/ab18.log
