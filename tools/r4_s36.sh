#!/bin/bash
# r4 s36: shapes near 16 x 2 over the driver's 20-frame window, four rounds
# (--steps 20 --warmup 5), bench lines interleaved over three rounds
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s36; mkdir -p $OUT
: > $OUT/shape.jsonl
for r in 1 2 3 4; do
for bf in 16:2 12:2 14:2 10:3 16:3; do
B=${bf%%:*}; F=${bf##*:}
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --batch $B --inflight $F --single-frame off --cpu-baseline off --critical-path off --reference-loop off > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'B': $B, 'F': $F, 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" >> $OUT/shape.jsonl
done
done
python - <<PY
import json, statistics, collections
d = collections.defaultdict(list)
for l in open("$OUT/shape.jsonl"):
    x = json.loads(l); d[(x['B'], x['F'])].append(x['value'])
for k, v in d.items(): print(k, round(statistics.median(v), 1), v)
PY
