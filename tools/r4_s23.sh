#!/bin/bash
# r4 s23: the committed kernel (side slots off; the hot instantiation's code
# is s19's): GPU tests, one frame alone with and without split tiles, the
# roofline session for this source and a plain bench line
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s23; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/split_sweep.py --split 0:16:1 0:16:1:L 32:16:1200 16:16:1200 64:16:1000 32:16:1600 0:16:1 32:16:1200 --inflight 4 --out $OUT/split_sweep.jsonl > $OUT/split_sweep.log 2>&1 || { tail -20 $OUT/split_sweep.log; exit 1; }
python -c "
import json
for l in open('$OUT/split_sweep.jsonl'): d=json.loads(l); print(d['split'], d['latency_ms'], d['identical'], d.get('ms_per_frame_F4'))"
SESSION=r4s23/roof bash tools/roofline_session.sh || exit 1
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:300])"
cp $OUT/roof/pmc_latest.json profiles/pmc_latest.json && cp $OUT/roof/traffic_latest.json profiles/traffic_latest.json
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('valu_issue_frac'), d['parity']['frame_sha_match'], json.dumps(d['config']['single_frame']))"
