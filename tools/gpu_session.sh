#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-s1}
mkdir -p "$OUT"
fatal() { case "$1" in 0|1|5) return 1;; *) return 0;; esac; }   # pytest 1 = failures, 5 = none collected
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 5 "$OUT/$name.log"
  return $rc
}
STEPS=${STEPS:-pytest,smoke,bench,prof}
if [[ $STEPS == *micro* ]]; then  # tools/microbench/tworay (built in the container)
  run tworay 120 tools/microbench/tworay || exit $?
  grep '^{' "$OUT/tworay.log" > "$OUT/tworay.json"
fi
if [[ $STEPS == *pytest* ]]; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}; rc=$?
  if fatal $rc; then echo "pytest fatal rc=$rc, stopping"; exit $rc; fi
fi
if [[ $STEPS == *smoke* ]]; then
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
fi
if [[ $STEPS == *bench* ]]; then
  run bench 600 python bench.py ${BENCH_ARGS:-} || exit $?
  grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
fi
if [[ $STEPS == *prof* ]]; then
  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --cpu-baseline off --critical-path off || exit $?
  find "$OUT/prof" -name "*stats*" -o -name "*kernel_stats*" | head -20
fi
if [[ $STEPS == *counters* ]]; then
  run counters 120 rocprofv3 -L || exit $?
fi
echo "session done"
