#!/bin/bash
# r4 s14: one rank's share of the headline frame on the one GPU (what each GPU
# of an N-GPU node renders), cost-balanced lists, the bench's pipeline:
# projected whole-job rates at N = 2 / 4 / 8 before the gather
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s14; mkdir -p $OUT
timeout -k 10 600 python tools/split_sweep.py --split 0:16:1 --balance cost --shard 0 1 --shard 0 2 --shard 0 4 --shard 0 8 --shard 7 8 --batch 8 16 --inflight 3 --frames 96 --out $OUT/shares.jsonl > $OUT/shares.log 2>&1 || { tail -20 $OUT/shares.log; exit 1; }
python - <<PY
import json
for l in open("$OUT/shares.jsonl"):
    d = json.loads(l); n = int(d["shard"].split("/")[1]); t = d["ms_per_frame_F3"]
    print(d["shard"], "B", d["batch"], "ms/frame", t, "projected Mpix/s", round(1920 * 1080 / t / 1e3, 1), "latency", d["latency_ms"])
PY
