#!/bin/bash
# r4 s38: 7 integrate waves per SIMD (w7: 72 VGPRs, 9 spills) against 6 in
# the 16 x 2 pipeline (96 frames) and the 8 x 3 one (48 frames)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s38; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
L="$V/libsr_cur.so $V/libsr_w7.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --batch 16 --inflight 2 --frames 96 --rounds 6 > $OUT/ab_tp16.log 2>&1 || { tail -20 $OUT/ab_tp16.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp16.log | tail -8
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 6 > $OUT/ab_tp8.log 2>&1 || { tail -20 $OUT/ab_tp8.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp8.log | tail -8
