#!/bin/bash
# round 5: camera records only in the CAM instantiation (parity suite, per-pass PMC, C3 bulk A/B
# against the build with a runtime record path in every shade instantiation and the build before)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05au; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/per_pass_pmc.sh $O/ppmc > $O/ppmc.txt 2>&1 || { echo "ppmc failed"; tail -5 $O/ppmc.txt; exit 1; }
head -12 $O/ppmc.txt
bash tools/gpu_ab.sh r05au_ab crec0=crec0 camv=camv camv2=camv2
