#!/bin/bash
# r4 s39: 6 / 7 / 8 integrate waves per SIMD, pipeline 16 x 2 (96 frames, 8
# rounds) and one frame alone
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s39; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
L="$V/libsr_cur.so $V/libsr_w7.so $V/libsr_w8.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --batch 16 --inflight 2 --frames 96 --rounds 8 > $OUT/ab_tp16.log 2>&1 || { tail -20 $OUT/ab_tp16.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp16.log | tail -12
timeout -k 10 300 python tools/ab_variants.py $L --rounds 6 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -12
