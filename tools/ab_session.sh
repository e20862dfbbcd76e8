#!/bin/bash
# GPU session for kernel A/B work: (optional) parity tests, then interleaved
# throughput (bench pipeline) and single-frame A/B of variant libraries.
#   LIBS="a b c" [PYTEST=1] SESSION=name bash tools/ab_session.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-ab}
mkdir -p "$OUT"
V=schwarzschild-raytracer_amd/lib/variants
L=""; for n in $LIBS; do L="$L $V/libsr_$n.so"; done
if [[ ${PYTEST:-1} == 1 ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --tb=short ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  grep -E "^E |FAIL|passed|failed" "$OUT/pytest_gpu.log" | head -30
  [[ $rc == 0 || $rc == 1 ]] || exit $rc
fi
timeout -k 10 500 python tools/ab_variants.py $L --throughput --rounds ${ROUNDS:-4} > "$OUT/ab_tp.log" 2>&1 || { tail -20 "$OUT/ab_tp.log"; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' "$OUT/ab_tp.log"
timeout -k 10 300 python tools/ab_variants.py $L --rounds ${ROUNDS:-4} > "$OUT/ab_single.log" 2>&1 || { tail -20 "$OUT/ab_single.log"; exit 1; }
grep -E '"lib|median_ms"|identical' "$OUT/ab_single.log"
echo "session done"
