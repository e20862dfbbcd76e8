#!/bin/bash
# bench.py over the driver's 20-frame window with several frames-per-launch /
# launches-in-flight settings, interleaved passes: [CONFIGS="8x3 10x3"] [PASSES=2] SESSION=sNN
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-sweep}; mkdir -p $OUT
for pass in $(seq ${PASSES:-2}); do
  for bf in ${CONFIGS:-8x3 10x2 10x3 7x3 5x4 4x5}; do  # frames per launch x launches in flight
    set -- ${bf/x/ }
    timeout -k 10 120 python bench.py --batch $1 --inflight $2 --cpu-baseline off --critical-path off --reference-loop off > $OUT/b$1_f$2_p$pass.log 2>&1 || exit $?
    python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['value'])" $OUT/b$1_f$2_p$pass.log $1 $2
  done
done | tee $OUT/sweep.txt
echo done
