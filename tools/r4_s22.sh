#!/bin/bash
# r4 s22: side slot with its ball and radius bound folded into the loop's
# q0 / ulo (7 spills instead of 13): GPU tests, A/B against head, section cycles
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s22; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_head.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -12
timeout -k 10 300 python tools/ab_variants.py $L --rounds 6 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -12
timeout -k 10 200 python tools/prof_waves.py $V/libsr_prof.so > $OUT/prof_full.json 2>&1 || { tail -5 $OUT/prof_full.json; exit 1; }
python - <<PY
import json
t = open("$OUT/prof_full.json").read(); p = json.loads(t[t.index("{"):])
tot = p["cycles_total_all_waves"]
print("total", tot, {k: round(v / tot, 4) for k, v in p["cycles_by_section_all_waves"].items()})
PY
