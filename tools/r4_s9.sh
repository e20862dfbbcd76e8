#!/bin/bash
# r4 s9: the shade kernel held to 5 / 6 / 8 waves per SIMD (96 / 80 / 64
# VGPRs, spilling) so it fits beside the integrate waves of the other
# streams; frames per launch x launches in flight with bench.py; a stream
# timeline of the default bench under --kernel-trace
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s9; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
L="schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_shade5.so $V/libsr_shade6.so $V/libsr_shade8.so"
timeout -k 10 400 python tools/ab_variants.py $L --throughput --rounds 4 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -12
for bf in "8 3" "8 2" "8 1" "16 2" "12 3" "6 4"; do
  set -- $bf
  timeout -k 10 200 python bench.py --batch $1 --inflight $2 --cpu-baseline off --critical-path off --reference-loop off --single-frame off > $OUT/bench_b$1_f$2.log 2>&1 || { tail -5 $OUT/bench_b$1_f$2.log; exit 1; }
  python -c "import json; d=json.loads([l for l in open('$OUT/bench_b$1_f$2.log') if l.startswith('{')][-1]); print('B $1 F $2', d['value'], d['ms_per_step'], d['parity']['frame_sha_match'])"
done
export GPU_MAX_HW_QUEUES=8
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python bench.py --cpu-baseline off --critical-path off --reference-loop off --single-frame off > $OUT/trace_bench.log 2>&1 || { tail -5 $OUT/trace_bench.log; exit 1; }
grep '^{' $OUT/trace_bench.log | tail -1 | cut -c1-300
