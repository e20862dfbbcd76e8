#!/bin/bash
# r4 s25: the look-ahead's factor for budgeted cylinders (SR_AHEAD_CYL 0 /
# 0.5 / 2 against 1): A/B and events
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s25; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
for n in stats stats_ahc0; do
timeout -k 10 200 python tools/stats_frame.py $V/libsr_$n.so > $OUT/$n.json 2>&1 || { tail -5 $OUT/$n.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/$n.json").read().strip().split("\n")[-1])
print("$n", "events", d["events"], "spent", [d.get("slot%d_spent" % j) for j in range(7)], "reached", [d.get("slot%d_reached" % j) for j in range(7)])
PY
done
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_ahc0.so $V/libsr_ahc05.so $V/libsr_ahc2.so"
timeout -k 10 500 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -16
