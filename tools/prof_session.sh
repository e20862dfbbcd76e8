#!/bin/bash
# SR_PROF section profile (tools/prof_waves.py) of variant libraries: NAMES="a b" SESSION=sNN
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-prof}; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
for n in $NAMES; do
  timeout -k 10 180 python tools/prof_waves.py $V/libsr_prof_$n.so > $OUT/prof_$n.json 2>&1 || exit $?
done
echo done
