#!/bin/bash
# r4 s17: where the integrate kernel's set-up and hand-off cycles go (SR_PROF
# sections 22 budget_init and 23 kernel start to integrate)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s17; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 200 python tools/prof_waves.py $V/libsr_prof.so > $OUT/prof_full.json 2>&1 || { tail -5 $OUT/prof_full.json; exit 1; }
python - <<PY
import json
t = open("$OUT/prof_full.json").read(); p = json.loads(t[t.index("{"):])
tot = p["cycles_total_all_waves"]
print({k: round(v / tot, 4) for k, v in p["cycles_by_section_all_waves"].items()})
print("tail_top", round(p["tail_top_all_waves"] / tot, 4), "budget_init", round(p["budget_init_all_waves"] / tot, 4), "ray_setup", round(p["ray_setup_all_waves"] / tot, 4), "rest", round(p["unaccounted_cycles_all_waves"] / tot, 4))
PY
OUT=gpurun_out/r4s18; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_cmi0.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -8
timeout -k 10 300 python tools/ab_variants.py $L --rounds 6 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -8
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats.so > $OUT/stats.json 2>&1 || { tail -5 $OUT/stats.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats.json").read().strip().split("\n")[-1])
print("events", d["events"], "wave_steps", d["wave_steps"], "cm", d["cm_wave_steps"], "spent", [d.get("slot%d_spent" % j) for j in range(7)])
PY
# the roofline session and a plain bench line at this kernel
SESSION=r4s18/roof bash tools/roofline_session.sh || exit 1
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:300])"
cp $OUT/roof/pmc_latest.json profiles/pmc_latest.json && cp $OUT/roof/traffic_latest.json profiles/traffic_latest.json
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('valu_issue_frac'), d['parity']['frame_sha_match'])"
