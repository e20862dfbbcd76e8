#!/bin/bash
# Throughput A/B of libsr variants on one GPU box: optional parity tests on a
# candidate variant (SR_LIB), then interleaved rounds of tools/split_sweep.py
# (headline frame, B frames per launch, F launches in flight) per variant.
#   LIBS="base p1" PARITY=p1 ROUNDS=3 SESSION=s26 bash tools/ab_throughput.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-abt}
mkdir -p "$OUT"
V=schwarzschild-raytracer_amd/lib/variants
for p in ${PARITY:-}; do
  SR_LIB=$PWD/$V/libsr_$p.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread > "$OUT/pytest_$p.log" 2>&1; rc=$?
  echo "parity $p rc=$rc: $(tail -n 1 "$OUT/pytest_$p.log")"
  [[ $rc == 0 ]] || exit $rc
done
for round in $(seq "${ROUNDS:-3}"); do
  for v in ${LIBS}; do
    timeout -k 10 300 python tools/split_sweep.py --lib $V/libsr_$v.so --batch ${BATCH:-8} \
      --inflight ${INFLIGHT:-3} --frames ${FRAMES:-48} ${SWEEP_ARGS:-} >> "$OUT/ab.jsonl" 2> "$OUT/err_$v.log" \
      || { echo "sweep $v rc=$?"; tail -n 20 "$OUT/err_$v.log"; exit 1; }
    tail -n 1 "$OUT/ab.jsonl"
  done
done
echo "session done"
