#!/bin/bash
# r4 s6: the new default kernel (no compact table): GPU tests, the shade
# kernel's marginal cost (constant-colour timing build), the roofline session
# (PMC passes, traffic, kernel stats, the headline bench line under --stats)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s6; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_variants.py schwarzschild-raytracer_amd/lib/libsr.so $V/libsr_constshade.so --throughput --rounds 4 > $OUT/ab_tp.log 2>&1 || { tail -20 $OUT/ab_tp.log; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' $OUT/ab_tp.log | tail -8
SESSION=r4s6/roof bash tools/roofline_session.sh || exit 1
python -c "import json; d=json.load(open('$OUT/roof/bench_stats.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:600])"
