#!/bin/bash
# r4 s33: the one-GPU headline shape 16 x 2 as bench.py's default: GPU tests,
# then the driver's command (--steps 20 --warmup 5) against the previous
# default shape (--batch 8 --inflight 3), alternating, four rounds
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s33; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
: > $OUT/driver_cmd.jsonl
for r in 1 2 3 4; do
for v in new old; do
X=""; [ $v = old ] && X="--batch 8 --inflight 3"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $X > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
grep '^{' $OUT/b.log > $OUT/b_${v}_$r.json
python -c "import json; d=json.load(open('$OUT/b_${v}_$r.json')); print(json.dumps({'round': $r, 'shape': '$v', 'B': d['config']['frames_per_launch'], 'F': d['config']['launches_in_flight'], 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'frac': d['roofline'].get('frac'), 'parity': d['parity']['frame_sha_match']}))" | tee -a $OUT/driver_cmd.jsonl
done
done
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); sf=d['config']['single_frame']; print('default', d['value'], d['ms_per_step'], d['config']['frames_per_launch'], d['config']['launches_in_flight'], d['roofline'].get('frac'), d['roofline'].get('valu_issue_frac'), d['parity']['frame_sha_match'], {k: v['ms_per_frame'] for k, v in sf.items()})"
