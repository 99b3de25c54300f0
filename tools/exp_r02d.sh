#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
X=$PWD/opengl-ray-tracing-framework_amd/lib/exp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python3 tools/ab_single.py --rounds 3 head=$X/librtamd_head.so p3=default p0=default:RT_FINISH_PASS=0 p2=default:RT_FINISH_PASS=2 p4=default:RT_FINISH_PASS=4 p5=default:RT_FINISH_PASS=5 fw2=$X/librtamd_fw2.so fw3=$X/librtamd_fw3.so > $O/ab_single.log 2>&1 || { tail -20 $O/ab_single.log; exit 1; }
tail -9 $O/ab_single.log
timeout -k 10 500 python3 tools/ab_proc.py --rounds 3 --whole base=$X/librtamd_head.so new=default > $O/ab_C3.log 2>&1 || { tail -20 $O/ab_C3.log; exit 1; }
tail -3 $O/ab_C3.log
