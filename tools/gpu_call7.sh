# env knobs re-checked on the rebuilt tree
export TMPDIR=/tmp
timeout -k 10 900 python3 tools/ab_proc.py --whole --rounds 3 base=default lds6=default:RT_LDS_STACK=6 lds10=default:RT_LDS_STACK=10 cam_dual=default:RT_TRACE_MODE0=3 chunk512=default:RT_POOL_CHUNK=512 > gpurun_out/ab7.log 2>&1 || { echo ab failed; tail -20 gpurun_out/ab7.log; exit 1; }
tail -6 gpurun_out/ab7.log
