#!/bin/bash
# r4 s24: the bench's single-frame figures timed round robin (split tiles,
# default launch, latency mode on three contexts): three bench runs
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s24; mkdir -p $OUT
for n in 1 2; do
timeout -k 10 300 python bench.py --cpu-baseline off --reference-loop off --critical-path off > $OUT/bench_quick$n.log 2>&1 || { tail -20 $OUT/bench_quick$n.log; exit 1; }
grep '^{' $OUT/bench_quick$n.log > $OUT/bench_quick$n.json
python -c "import json; d=json.load(open('$OUT/bench_quick$n.json')); sf=d['config']['single_frame']; print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), {k: v['ms_per_frame'] for k, v in sf.items()})"
done
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); sf=d['config']['single_frame']; print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('valu_issue_frac'), d['parity']['frame_sha_match'], {k: v['ms_per_frame'] for k, v in sf.items()}, d['cpu_baseline']['value'])"
