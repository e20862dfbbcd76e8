#!/bin/bash
# r4 s4: GPU tests on the current kernel (compact step table, no VGPR spills in
# the hot instantiation), A/B against the round-3 kernel, the LDS-state kernel
# with orbital-plane exclusion (xp), the same without the compact table (ct0)
# and without the exclusion (noxp); event counters; bench
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s4; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
L="$V/libsr_xp.so $V/libsr_ct0.so $V/libsr_noxp.so schwarzschild-raytracer_amd/lib/libsr.so"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/ab_variants.py $L --throughput --rounds 4 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -10
timeout -k 10 300 python tools/ab_variants.py $L --rounds 4 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -10
for s in stats stats_noxp stats_nc; do
  timeout -k 10 200 python tools/stats_frame.py $V/libsr_$s.so > $OUT/$s.json 2>&1 || exit 1
done
python - <<PY
import json
for f in ("stats", "stats_noxp", "stats_nc"):
    d = json.loads(open("$OUT/%s.json" % f).read().strip().split("\n")[-1])
    print(f, "events", d.get("events"), "wave_steps", d.get("wave_steps"), "clock", d.get("clock_ghz"), "spent", [d.get("slot%d_spent" % j) for j in range(7)])
PY
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['config'].get('single_frame'))"
