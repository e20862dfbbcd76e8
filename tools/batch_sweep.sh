#!/bin/bash
# bench.py over the driver's 20-frame window with several frames-per-launch /
# launches-in-flight settings, two interleaved passes: SESSION=sNN
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-sweep}; mkdir -p $OUT
for pass in 1 2; do
  for bf in ${CONFIGS:-"8 3" "10 2" "10 3" "7 3" "5 4" "20 1" "4 5"}; do
    set -- $bf
    timeout -k 10 120 python bench.py --batch $1 --inflight $2 --cpu-baseline off --critical-path off --reference-loop off > $OUT/b$1_f$2_p$pass.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'])" $OUT/b$1_f$2_p$pass.log $1 $2
  done
done | tee $OUT/sweep.txt
echo done
