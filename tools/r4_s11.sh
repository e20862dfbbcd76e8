#!/bin/bash
# r4 s11: would an orbital-plane exclusion of the cylinder remove its
# re-anchors? (SR_STATS_XCYL probe build: per re-anchor, whether every lane
# that spent the cylinder's budget has a plane 3.6 / 5 / 8 from its centre
# and no near-axis chords)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s11; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 200 python tools/stats_frame.py $V/libsr_xcyl.so --xcyl > $OUT/stats_xcyl.json 2>&1 || { tail -5 $OUT/stats_xcyl.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats_xcyl.json").read().strip().split("\n")[-1])
print("events", d["events"], "spent", [d.get("slot%d_spent" % j) for j in range(7)], "xcyl", d["xcyl"])
PY
