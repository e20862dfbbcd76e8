#!/bin/bash
# r4 s40: batched launches of the small instantiation at 7 waves per SIMD
# (SR_BATCH_WAVES): GPU tests, A/B against head in the 16 x 2 pipeline, the
# driver's command alternating with head's library, the roofline session
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s40; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_head.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --batch 16 --inflight 2 --frames 96 --rounds 8 > $OUT/ab_tp16.log 2>&1 || { tail -20 $OUT/ab_tp16.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp16.log | tail -8
: > $OUT/driver_cmd.jsonl
for r in 1 2 3 4; do
for v in new head; do
X=""; [ $v = head ] && X="SR_LIB=$V/libsr_head.so"
env $X timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --single-frame off --cpu-baseline off --critical-path off --reference-loop off > $OUT/b.log 2>&1 || { tail -20 $OUT/b.log; exit 1; }
grep '^{' $OUT/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'round': $r, 'lib': '$v', 'value': d['value'], 'ms_per_step': d['ms_per_step']}))" | tee -a $OUT/driver_cmd.jsonl
done
done
SESSION=r4s40/roof bash tools/roofline_session.sh > $OUT/roof.log 2>&1 || { tail -20 $OUT/roof.log; exit 1; }
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:400])"
