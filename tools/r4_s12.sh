#!/bin/bash
# r4 s12: the cylinder's plane window (SR_CYL_PLANE): GPU tests, A/B against
# the same kernel without it (nocp), event counters and section cycles
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s12; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_nocp.so $V/libsr_qp.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 5 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -8
timeout -k 10 300 python tools/ab_variants.py $L --rounds 5 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -8
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats.so > $OUT/stats.json 2>&1 || { tail -5 $OUT/stats.json; exit 1; }
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats_qp.so > $OUT/stats_qp.json 2>&1 || { tail -5 $OUT/stats_qp.json; exit 1; }
timeout -k 10 200 python tools/prof_waves.py $V/libsr_prof.so > $OUT/prof_full.json 2>&1 || { tail -5 $OUT/prof_full.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats.json").read().strip().split("\n")[-1])
print("events", d["events"], "spent", [d.get("slot%d_spent" % j) for j in range(7)], "intervals", d["event_interval_steps"])
d = json.loads(open("$OUT/stats_qp.json").read().strip().split("\n")[-1])
print("qp events", d["events"], "spent", [d.get("slot%d_spent" % j) for j in range(7)])
t = open("$OUT/prof_full.json").read(); p = json.loads(t[t.index("{"):])
c = p["cycles_by_section_all_waves"]; tot = p["cycles_total_all_waves"]
print({k: round(v / tot, 4) for k, v in c.items()}, "tail_top", round(p["tail_top_all_waves"] / tot, 4), "tot", tot)
PY
