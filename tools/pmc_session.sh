#!/bin/bash
# PMC counter passes (each its own rocprofv3 run, kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-pmc}
mkdir -p "$OUT"
ARGS=${PROF_ARGS:-}
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  echo "== pass $i: $line"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $line -d "$OUT/p$i" -o run --output-format csv -- python tools/prof_frame.py --frames 2 $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  case $rc in 0) ;; *) echo "stopping"; exit $rc;; esac
done <<< "${PASSES:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH
FETCH_SIZE
WRITE_SIZE}"
echo done
