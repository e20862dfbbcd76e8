#!/bin/bash
# GPU session: parity tests, then interleaved A/B of variant libraries, then bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-ab}
mkdir -p "$OUT"
V=schwarzschild-raytracer_amd/lib/variants
if [[ ${SKIP_TESTS:-0} != 1 ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -rA > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  tail -n 3 "$OUT/pytest_gpu.log"
  [[ $rc == 0 ]] || { echo "pytest rc=$rc"; exit $rc; }
fi
for scene in ${SCENES:-tex untex}; do
  timeout -k 10 600 python tools/ab_variants.py ${LIBS} --scene $scene --rounds ${ROUNDS:-4} > "$OUT/ab_$scene.log" 2>&1 || { echo "ab rc=$?"; tail -n 20 "$OUT/ab_$scene.log"; exit 1; }
  tail -n 12 "$OUT/ab_$scene.log"
done
if [[ ${BENCH:-1} == 1 ]]; then
  timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1 || { echo "bench rc=$?"; tail -n 20 "$OUT/bench.log"; exit 1; }
  grep '^{' "$OUT/bench.log" > "$OUT/bench.json"; cat "$OUT/bench.json"
fi
echo "session done"
