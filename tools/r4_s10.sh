#!/bin/bash
# r4 s10: the small-LDS kernel: GPU tests, event counters (SR_STATS), section
# cycles (SR_PROF), the C++ node driver against bench.py, the roofline session
# (PMC passes, traffic, the bench line under --stats) and a plain bench run
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s10; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats.so > $OUT/stats.json 2>&1 || { tail -5 $OUT/stats.json; exit 1; }
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats_nc.so > $OUT/stats_nc.json 2>&1 || { tail -5 $OUT/stats_nc.json; exit 1; }
python - <<PY
import json
d = json.loads(open("$OUT/stats.json").read().strip().split("\n")[-1])
print("events", d["events"], "wave_steps", d["wave_steps"], "spent", [d.get("slot%d_spent" % j) for j in range(7)], "handoff", d["handoff"])
PY
timeout -k 10 200 python tools/prof_waves.py $V/libsr_prof.so > $OUT/prof_full.json 2>&1 || { tail -5 $OUT/prof_full.json; exit 1; }
python - <<PY
import json
t = open("$OUT/prof_full.json").read(); d = json.loads(t[t.index("{"):])
c = d["cycles_by_section_all_waves"]; tot = d["cycles_total_all_waves"]
print({k: round(v / tot, 4) for k, v in c.items()}, "tail_top", round(d["tail_top_all_waves"] / tot, 4), "events", d["events_all_waves"])
PY
timeout -k 10 500 python -u tools/cpp_driver_bench.py --rounds 3 --frames 96 > $OUT/cpp_vs_bench.jsonl 2> $OUT/cpp_vs_bench.err; rc=$?; tail -2 $OUT/cpp_vs_bench.jsonl; [ $rc -eq 0 ] || exit $rc
SESSION=r4s10/roof bash tools/roofline_session.sh || exit 1
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:400])"
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), json.dumps(d['config']['single_frame'])[:500])"
