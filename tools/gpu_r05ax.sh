#!/bin/bash
# round 5 final evidence on HEAD (tests, profiles, bench, interactive), then the small-shade A/B
set -o pipefail
export TMPDIR=/tmp
TAG=r05_C3 bash tools/round_gpu.sh || exit 1
bash tools/gpu_r05aw.sh
