#!/bin/bash
# r4 s29: in-plane planar budgets (SR_PLANE2D) with the look-ahead re-swept
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s29; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_head.so $V/libsr_p2a15.so $V/libsr_p2a25.so $V/libsr_p2t075.so $V/libsr_p2t15.so"
timeout -k 10 600 python tools/ab_variants.py $L --throughput --rounds 8 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -24
