#!/bin/bash
# r4 s3: GPU tests on the LDS-budget kernel, A/B against the round-3 kernel, bench
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s3; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 500 python tools/ab_variants.py $V/libsr_r3.so $V/libsr_lds.so $V/libsr_lds2.so $V/libsr_lds_u2.so --throughput --rounds 4 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -8
timeout -k 10 300 python tools/ab_variants.py $V/libsr_r3.so $V/libsr_lds.so $V/libsr_lds2.so $V/libsr_lds_u2.so --rounds 4 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -8
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['config']['single_frame'])"
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats_nc.so > $OUT/stats_nocount.json 2>&1; python -c "import json; d=json.loads(open('$OUT/stats_nocount.json').read().strip().split('\n')[-1]); print('clock', d.get('clock_ghz'), 'timeline_us', d['timeline_us'])"
timeout -k 10 200 python tools/stats_frame.py $V/libsr_stats.so > $OUT/stats.json 2>&1; python -c "import json; d=json.loads(open('$OUT/stats.json').read().strip().split('\n')[-1]); print('events', d['events'], 'wave_steps', d['wave_steps'])"
