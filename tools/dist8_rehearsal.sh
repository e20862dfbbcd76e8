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
# the flyby at N = 8: lists re-priced every 3 launches (default) and frame-0 lists kept
for rp in -1 0; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
    --master-port 29518 bench.py --gpus 8 --steps 40 --warmup 3 --dist-backend gloo --camera flyby --reprice $rp \
    --cpu-baseline off > "$OUT/bench8_flyby_rp$rp.log" 2>&1 || { echo "bench8 flyby rc=$?"; tail -n 30 "$OUT/bench8_flyby_rp$rp.log"; exit 1; }
  grep '^{' "$OUT/bench8_flyby_rp$rp.log" > "$OUT/bench8_flyby_rp$rp.json"
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['value'], json.dumps(d['config']['balance']))" "$OUT/bench8_flyby_rp$rp.json"
done
echo "session done"
