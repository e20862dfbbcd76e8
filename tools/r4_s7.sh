#!/bin/bash
# r4 s7: SR_PROF section cycles (whole frame, critical band)


cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s7; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 200 python tools/prof_waves.py $V/libsr_prof.so > $OUT/prof_full.json 2>&1 || { tail -5 $OUT/prof_full.json; exit 1; }
tail -c 1500 $OUT/prof_full.json
timeout -k 10 200 python tools/prof_waves.py $V/libsr_prof.so --rows 704 720 > $OUT/prof_band.json 2>&1 || { tail -5 $OUT/prof_band.json; exit 1; }
tail -c 800 $OUT/prof_band.json
timeout -k 10 60 rocprofv3 -L > $OUT/list_avail.txt 2>&1; echo "list rc=$?"
grep -i -A12 'pc sampl\|pc_sampl' $OUT/list_avail.txt | head -40
