#!/bin/bash
# r4 s37: split tiles in the throughput pipeline (16 x 2) over the driver's
# 20-frame window and over 96 frames, interleaved with the default
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s37; mkdir -p $OUT
: > $OUT/split.jsonl
for r in 1 2 3; do
for K in 20 96; do
for sp in 0 32:16:1200 64:16:1000 128:16:800; do
timeout -k 10 200 python bench.py --steps $K --warmup 5 --split $sp --single-frame off --cpu-baseline off --critical-path off --reference-loop off > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'K': $K, 'split': '$sp', 'value': d['value'], 'ms_per_step': d['ms_per_step'], 'parity': d['parity']['frame_sha_match']}))" >> $OUT/split.jsonl
done
done
done
python - <<PY
import json, statistics, collections
d = collections.defaultdict(list)
for l in open("$OUT/split.jsonl"):
    x = json.loads(l); d[(x['K'], x['split'])].append(x['value']); assert x['parity']
for k, v in sorted(d.items()): print(k, round(statistics.median(v), 1), v)
PY
