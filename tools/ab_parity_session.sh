#!/bin/bash
# GPU session for a kernel change: the GPU tests on variant library $TEST
# (SR_LIB), interleaved A/B timing of $LIBS (tools/ab_session.sh) and the
# SR_STATS counters of $STATS (tools/stats_frame.py).
#   TEST=name LIBS="a b" STATS="a b" SESSION=sNN bash tools/ab_parity_session.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-ab}; mkdir -p $OUT
V=$PWD/schwarzschild-raytracer_amd/lib/variants
if [[ -n $TEST ]]; then
  SR_LIB=$V/libsr_$TEST.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_$TEST.log 2>&1; rc=$?
  tail -12 $OUT/pytest_$TEST.log
  [[ $rc == 0 || $rc == 1 ]] || exit $rc
fi
for n in $STATS; do
  timeout -k 10 180 python tools/stats_frame.py $V/libsr_stats_$n.so > $OUT/stats_$n.json 2>&1 || exit $?
  python -c "import json,sys; t=open('$OUT/stats_$n.json').read(); d=json.loads(t[t.index('{'):]); print('$n', {k: d[k] for k in d if k.startswith(('events','slot')) and 'reached' not in k})"
done
if [[ -n $LIBS ]]; then PYTEST=0 bash tools/ab_session.sh || exit $?; fi
echo "session done"
