#!/bin/bash
# r4 s18: the cylinder-plane fast loop testing the chord direction once per
# three-step iteration when every lane is in a black-hole u window (CMV 2):
# GPU tests, A/B against the per-step test (cmi0), events
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s18; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_cmi0.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -8
timeout -k 10 300 python tools/ab_variants.py $L --rounds 6 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -8
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats.so > $OUT/stats.json 2>&1 || { tail -5 $OUT/stats.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats.json").read().strip().split("\n")[-1])
print("events", d["events"], "wave_steps", d["wave_steps"], "cm", d["cm_wave_steps"], "spent", [d.get("slot%d_spent" % j) for j in range(7)])
PY
