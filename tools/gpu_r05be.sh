#!/bin/bash
# round 5: pass-1 shade sort keyed by hit material too (C3 bulk A/B)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_ab.sh r05be_ab mk1=mk1 mk4=mk4
