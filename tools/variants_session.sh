#!/bin/bash
# Bench lines for the non-headline BASELINE.json configs and the SURVEY §8(f)
# row-3 variants (split modes 2/3, noise mask 0.75, reference loop without
# culling, the max-capacity scene and the press-R overlay at config 2's size), and the headline with single-frame launches and a flyby camera. One bench.py process per line, each under its own time limit;
# a failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-variants}
mkdir -p "$OUT"
run() {  # name timeout bench-args...
  local name=$1 t=$2; shift 2
  echo "== $name: bench.py $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$t" python bench.py --cpu-baseline off --critical-path off "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  grep '^{' "$OUT/$name.log" >> "$OUT/variants.jsonl"
  return $rc
}
run headline 180 --steps 20 --warmup 3 || exit $?
run headline_b1 180 --batch 1 --inflight 4 --steps 20 --warmup 3 || exit $?
run flyby 180 --camera flyby --steps 20 --warmup 3 || exit $?
run flyby_b1 180 --camera flyby --batch 1 --inflight 4 --steps 20 --warmup 3 || exit $?
run small 180 --workload small --steps 20 --warmup 3 || exit $?
run 4k 240 --workload 4k --steps 5 --warmup 1 || exit $?
run 8k 300 --workload 8k --steps 2 --warmup 1 || exit $?
run half_width 180 --mode half_width --steps 20 --warmup 3 || exit $?
run half_height 180 --mode half_height --steps 20 --warmup 3 || exit $?
run flat 180 --mode flat --steps 20 --warmup 3 || exit $?
run noise075 180 --percent-black 0.75 --steps 20 --warmup 3 || exit $?
run stress 240 --workload small --scene stress --steps 20 --warmup 3 || exit $?
run testray 300 --workload small --test-ray on --single-frame off --steps 20 --warmup 3 || exit $?
run no_cull 300 --no-cull --steps 3 --warmup 1 || exit $?
echo "session done"
