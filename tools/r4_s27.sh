#!/bin/bash
# r4 s27: in-plane distance budgets for planar slots (SR_PLANE2D): GPU tests,
# events against the previous kernel, A/B
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s27; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for n in stats stats_head; do
timeout -k 10 200 python tools/stats_frame.py $V/libsr_$n.so > $OUT/$n.json 2>&1 || { tail -5 $OUT/$n.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/$n.json").read().strip().split("\n")[-1])
print("$n", "events", d["events"], "spent", [d.get("slot%d_spent" % j) for j in range(7)], "reached", [d.get("slot%d_reached" % j) for j in range(7)])
PY
done
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_head.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -8
timeout -k 10 300 python tools/ab_variants.py $L --rounds 6 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -8
