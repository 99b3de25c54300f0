#!/bin/bash
# Build the committed (HEAD or $REV) librtamd.so as lib/exp/librtamd_${NAME:-head}.so for A/B runs.
set -e
REV=${REV:-HEAD}
D=$(mktemp -d)
git archive $REV opengl-ray-tracing-framework_amd include | tar -x -C $D
make -s -C $D/opengl-ray-tracing-framework_amd lib/librtamd.so
mkdir -p opengl-ray-tracing-framework_amd/lib/exp
cp $D/opengl-ray-tracing-framework_amd/lib/librtamd.so opengl-ray-tracing-framework_amd/lib/exp/librtamd_${NAME:-head}.so
rm -rf $D
