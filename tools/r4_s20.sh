#!/bin/bash
# r4 s20: SR_STATS_PLANE probe - how many budget events only planar slots'
# chords that stay off their acceptance slab triggered
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s20; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats_plane.so --plane > $OUT/stats_plane.json 2>&1 || { tail -5 $OUT/stats_plane.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats_plane.json").read().strip().split("\n")[-1])
print("events", d["events"], d["plane"], d["event_interval_steps"])
PY
