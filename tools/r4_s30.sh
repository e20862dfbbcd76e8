#!/bin/bash
# r4 s30: the roofline session and a plain bench line with in-plane planar
# budgets (SR_PLANE2D)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s30; mkdir -p $OUT
SESSION=r4s30/roof bash tools/roofline_session.sh || exit 1
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:300])"
cp $OUT/roof/pmc_latest.json profiles/pmc_latest.json && cp $OUT/roof/traffic_latest.json profiles/traffic_latest.json
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); sf=d['config']['single_frame']; print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('valu_issue_frac'), d['parity']['frame_sha_match'], {k: v['ms_per_frame'] for k, v in sf.items()})"
