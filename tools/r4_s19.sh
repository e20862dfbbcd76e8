#!/bin/bash
# r4 s19: budget_init with slot j+1's record loaded while slot j is worked on
# and the orbital-plane exclusion folded into that pass: GPU tests, A/B
# against the previous kernel (head), section cycles of both, roofline session
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s19; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_head.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -8
timeout -k 10 300 python tools/ab_variants.py $L --rounds 6 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -8
for n in prof prof_head; do
timeout -k 10 200 python tools/prof_waves.py $V/libsr_$n.so > $OUT/${n}_full.json 2>&1 || { tail -5 $OUT/${n}_full.json; exit 1; }
python - <<PY
import json
t = open("$OUT/${n}_full.json").read(); p = json.loads(t[t.index("{"):])
tot = p["cycles_total_all_waves"]
print("$n", "total", tot, "budget_init", round(p["budget_init_all_waves"] / tot, 4), "ray_setup", round(p["ray_setup_all_waves"] / tot, 4))
PY
done
SESSION=r4s19/roof bash tools/roofline_session.sh || exit 1
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:300])"
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('valu_issue_frac'), d['parity']['frame_sha_match'])"
