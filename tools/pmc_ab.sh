#!/bin/bash
# PMC comparison of libsr variants: one rocprofv3 --pmc pass per (variant, pass),
# kernel trace only. VARIANTS="name ..." (lib/variants/libsr_<name>.so), PASSES as in pmc_session.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-pmcab}
mkdir -p "$OUT"
PASSES=${PASSES:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"}
for v in ${VARIANTS}; do
  i=0
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    export SR_LIB=schwarzschild-raytracer_amd/lib/variants/libsr_$v.so
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $line -d "$OUT/$v/p$i" -o run --output-format csv -- python tools/prof_frame.py --frames 2 ${PROF_ARGS:-} > "$OUT/$v.p$i.log" 2>&1
    rc=$?
    echo "$v pass $i rc=$rc"
    [ $rc == 0 ] || exit $rc
  done <<< "$PASSES"
  python tools/pmc_summary.py "$OUT/$v"
done
