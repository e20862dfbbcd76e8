#!/bin/bash
# r4 s21: side slots (SR_SIDE): planar slots' budgets replaced by per-step
# side tests at events that only planar slots triggered: GPU tests, events,
# A/B against the previous kernel (head) and two side slots (side2)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s21; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats_plane.so --plane > $OUT/stats_plane.json 2>&1 || { tail -5 $OUT/stats_plane.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats_plane.json").read().strip().split("\n")[-1])
print("events", d["events"], "wave_steps", d["wave_steps"], d["plane"], d["side"], d["event_interval_steps"])
PY
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_head.so $V/libsr_side2.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -12
timeout -k 10 300 python tools/ab_variants.py $L --rounds 6 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -12
