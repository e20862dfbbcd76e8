#!/bin/bash
# r4 s13: knob sweep at the current kernel (look-ahead, near-wave clearance,
# priority blocks, coasting, fast-loop unroll 2) in the pipeline A/B, then the
# bench lines of the other configurations (tools/variants_session.sh)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s13; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
L="schwarzschild-raytracer_amd/lib/libsr.so"
for n in ah15 ah25 aht075 aht15 near075 near15 prio0 coast0 fu2 res64; do L="$L $V/libsr_$n.so"; done
timeout -k 10 600 python tools/ab_variants.py $L --throughput --rounds 3 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
python - <<PY
import json, re
t = open("$OUT/ab_tp.log").read()
i = t.rfind("{\n"); d = json.loads(t[t.index("{"):]) if t.strip().startswith("{") else None
PY
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -30
SESSION=r4s13/variants bash tools/variants_session.sh || exit 1
python - <<PY
import json
for l in open("$OUT/variants/variants.jsonl"):
    d = json.loads(l); c = d["config"]
    print(c.get("workload"), c.get("mode", ""), c.get("camera"), d["value"], d["ms_per_step"], c.get("frames_per_launch"), c.get("launches_in_flight"), c.get("frame_latency_ms"))
PY
