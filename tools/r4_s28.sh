#!/bin/bash
# r4 s28: in-plane planar budgets with the cylinder's plane window (p2c) and
# the spheres' and boxes' (p2cq): events and A/B against p2 alone and head
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s28; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
for n in stats_p2c stats_p2cq; do
timeout -k 10 200 python tools/stats_frame.py $V/libsr_$n.so > $OUT/$n.json 2>&1 || { tail -5 $OUT/$n.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/$n.json").read().strip().split("\n")[-1])
print("$n", "events", d["events"], "spent", [d.get("slot%d_spent" % j) for j in range(7)])
PY
done
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_head.so $V/libsr_p2c.so $V/libsr_p2cq.so"
timeout -k 10 500 python tools/ab_variants.py $L --throughput --rounds 8 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -16
