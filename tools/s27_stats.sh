# SR_STATS / SR_PROF counters of two kernels (before / after a change)
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-s27}; mkdir -p $OUT
V=schwarzschild-raytracer_amd/lib/variants
for n in ${NAMES:-head ball}; do
  timeout -k 10 180 python tools/stats_frame.py $V/libsr_stats_$n.so > $OUT/stats_$n.json 2>&1 || exit $?
  timeout -k 10 180 python tools/prof_waves.py $V/libsr_prof_$n.so > $OUT/prof_$n.json 2>&1 || exit $?
done
echo done
