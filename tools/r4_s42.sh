#!/bin/bash
# r4 s42: stream priorities of the two launch slots (SR_BENCH_STREAM_PRIO: a
# timing-only bench.py option of that session, removed after it),
# 96 and 20 frames, interleaved with the default
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s42; mkdir -p $OUT
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
: > $OUT/prio.jsonl
for r in 1 2 3; do
for K in 96 20; do
for pr in none -1,0 0,0 -1,-1; do
X=""; [ $pr != none ] && X="SR_BENCH_STREAM_PRIO=$pr"
env $X timeout -k 10 200 python bench.py --steps $K --warmup 5 --single-frame off --cpu-baseline off --critical-path off --reference-loop off > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'K': $K, 'prio': '$pr', 'value': d['value']}))" >> $OUT/prio.jsonl
done
done
done
python - <<PY
import json, statistics, collections
d = collections.defaultdict(list)
for l in open("$OUT/prio.jsonl"):
    x = json.loads(l); d[(x['K'], x['prio'])].append(x['value'])
for k, v in sorted(d.items()): print(k, round(statistics.median(v), 1), v)
PY
