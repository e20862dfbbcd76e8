#!/bin/bash
# r4 s8: the small instantiation with its own LDS layout (6 slots, 1 cylinder:
# 17 rows, 4.5 KiB per wave, no VGPR spills): GPU tests; occupancy timing
# builds with the same layout (lds17w6/w7/w8: 6 / 7 / 8 waves per SIMD) against
# it; one frame alone with split tiles and the latency mode (split_sweep)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s8; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_ct0.so $V/libsr_lds17w6.so $V/libsr_lds17w7.so $V/libsr_lds17w8.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 4 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -15
timeout -k 10 300 python tools/ab_variants.py $L --rounds 4 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -15
timeout -k 10 400 python tools/split_sweep.py --split 0:16:1 0:16:1:L 64:16:1000 64:16:1000:L 128:16:1000 32:16:1200 64:4:1000 --inflight 4 --out $OUT/split_sweep.jsonl > $OUT/split_sweep.log 2>&1 || { tail -20 $OUT/split_sweep.log; exit 1; }
python -c "
import json
for l in open('$OUT/split_sweep.jsonl'): d=json.loads(l); print(d['split'], d['latency_ms'], d['identical'], d.get('ms_per_frame_F4'))"
