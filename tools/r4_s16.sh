#!/bin/bash
# r4 s16: the final kernel of the round: GPU tests, event counters, section
# cycles, the C++ node driver against bench.py, the roofline session and a
# plain bench run
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s16; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats.so > $OUT/stats.json 2>&1 || { tail -5 $OUT/stats.json; exit 1; }
timeout -k 10 200 python tools/prof_waves.py $V/libsr_prof.so > $OUT/prof_full.json 2>&1 || { tail -5 $OUT/prof_full.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats.json").read().strip().split("\n")[-1])
print("events", d["events"], "wave_steps", d["wave_steps"], "cm", d["cm_wave_steps"], "spent", [d.get("slot%d_spent" % j) for j in range(7)])
t = open("$OUT/prof_full.json").read(); p = json.loads(t[t.index("{"):])
c = p["cycles_by_section_all_waves"]; tot = p["cycles_total_all_waves"]
print({k: round(v / tot, 4) for k, v in c.items()}, "tail_top", round(p["tail_top_all_waves"] / tot, 4), "unacc", round(p["unaccounted_cycles_all_waves"] / tot, 4))
PY
timeout -k 10 500 python -u tools/cpp_driver_bench.py --rounds 3 --frames 96 > $OUT/cpp_vs_bench.jsonl 2> $OUT/cpp_vs_bench.err; rc=$?; tail -1 $OUT/cpp_vs_bench.jsonl; [ $rc -eq 0 ] || exit $rc
SESSION=r4s16/roof bash tools/roofline_session.sh || exit 1
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:400])"
cp $OUT/roof/pmc_latest.json profiles/pmc_latest.json && cp $OUT/roof/traffic_latest.json profiles/traffic_latest.json
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic'), json.dumps(d['config']['single_frame'])[:300])"
