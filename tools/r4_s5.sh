#!/bin/bash
# r4 s5: the fast loop's u' chain kept before the exit branch (dun), with the
# compact table and without (ct0dun), against HEAD (head) and the s4 winner
# without the compact table (ct0): interleaved throughput and one frame alone
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s5; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
L="$V/libsr_ct0.so $V/libsr_head.so $V/libsr_dun.so $V/libsr_ct0dun.so"
timeout -k 10 500 python tools/ab_variants.py $L --throughput --rounds 4 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -12
timeout -k 10 300 python tools/ab_variants.py $L --rounds 4 > $OUT/ab_single.log 2>&1 || { tail -20 $OUT/ab_single.log; exit 1; }
grep -E '"lib|median_ms"|identical' $OUT/ab_single.log | tail -12
