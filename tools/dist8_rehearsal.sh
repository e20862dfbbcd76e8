#!/bin/bash
# 8 ranks sharing the one leased GPU: the multi-rank GPU tests (incl. world 8)
# and the headline bench command as the driver launches it at N = 8, over gloo
# with host-staged tiles (RCCL needs one GPU per rank). Each step has its own
# time limit; a failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-dist8}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py -m gpu -x -v --timeout 400 --timeout-method thread > "$OUT/pytest_dist.log" 2>&1 || { echo "pytest rc=$?"; tail -n 30 "$OUT/pytest_dist.log"; exit 1; }
tail -n 6 "$OUT/pytest_dist.log"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --steps 20 --warmup 3 --dist-backend gloo > "$OUT/bench8.log" 2>&1 \
  || { echo "bench8 rc=$?"; tail -n 30 "$OUT/bench8.log"; exit 1; }
grep '^{' "$OUT/bench8.log" > "$OUT/bench8.json"; cat "$OUT/bench8.json"
# the flyby at N = 8: the default (auto: cyclic rows for a moving camera),
# cost lists re-priced every 3 launches, and the frame-0 cost lists kept
for v in "auto -1" "cost -1" "cost 0"; do
  set -- $v
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 8 --steps 40 --warmup 3 --dist-backend gloo --camera flyby --balance $1 \
    --reprice $2 --cpu-baseline off > "$OUT/bench8_flyby_$1_rp$2.log" 2>&1 || { echo "bench8 flyby rc=$?"; tail -n 30 "$OUT/bench8_flyby_$1_rp$2.log"; exit 1; }
  grep '^{' "$OUT/bench8_flyby_$1_rp$2.log" > "$OUT/bench8_flyby_$1_rp$2.json"
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[1], d['value'], c['balance_policy'], c['last_camera_max_over_mean'], (c['balance'] or {}).get('reprice_choices'))" "$OUT/bench8_flyby_$1_rp$2.json"
done
# the driver's own shape: bench.py --gpus 8 without a launcher (it spawns its ranks)
timeout -k 10 400 python bench.py --gpus 8 --steps 20 --warmup 3 --dist-backend gloo --cpu-baseline off > "$OUT/bench8_spawn.log" 2>&1 \
  || { echo "bench8 spawn rc=$?"; tail -n 30 "$OUT/bench8_spawn.log"; exit 1; }
grep '^{' "$OUT/bench8_spawn.log" > "$OUT/bench8_spawn.json"
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('spawned', d['n_gpus'], d['config']['world_size'], d['parity'])" "$OUT/bench8_spawn.json"
echo "session done"
