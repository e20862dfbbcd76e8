#!/bin/bash
# Roofline evidence for the headline command, on the GPU box (one gpurun call):
#   1. FLOP-counter calibration (tools/microbench/flops_calib, known work)
#   2. PMC passes over bench.py itself (four frames in flight, the headline
#      config), each its own rocprofv3 run with --kernel-trace only
#   3. rocprofv3 --kernel-trace --stats of the same bench command (kernel_ms
#      agreement) and its JSON line
#   4. tools/pmc_flops.py / tools/traffic_json.py -> $OUT/pmc_latest.json,
#      $OUT/traffic_latest.json (copied into profiles/ by hand)
# Every GPU step has its own time limit; a failure ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-roof}
mkdir -p "$OUT"
BENCH="bench.py --steps ${PMC_STEPS:-8} --warmup 4 --cpu-baseline off --critical-path off --reference-loop off ${BENCH_ARGS:-}"
# HIP reads GPU_MAX_HW_QUEUES before bench.py runs when a profiler preloads it
export GPU_MAX_HW_QUEUES=8
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -n 3 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
}
FLOPS="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_WAVES"
step calib 60 rocprofv3 --kernel-trace --pmc $FLOPS -d "$OUT/calib" -o run --output-format csv -- tools/microbench/flops_calib
step p1 300 rocprofv3 --kernel-trace --pmc $FLOPS -d "$OUT/p1" -o run --output-format csv -- python $BENCH
step p2 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE -d "$OUT/p2" -o run --output-format csv -- python $BENCH
step p3 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/p3" -o run --output-format csv -- python $BENCH
step p4 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/p4" -o run --output-format csv -- python $BENCH
python tools/pmc_flops.py --calib "$OUT/calib" --frame "$OUT/p1" "$OUT/p2" --out "$OUT/pmc_latest.json" \
    --source "$OUT (tools/roofline_session.sh)" ${SIZE_ARGS:-} > "$OUT/pmc_flops.log" 2>&1 || { cat "$OUT/pmc_flops.log"; exit 1; }
cat "$OUT/pmc_flops.log"
python tools/traffic_json.py --frame "$OUT/p3" "$OUT/p4" --out "$OUT/traffic_latest.json" ${SIZE_ARGS:-} > "$OUT/traffic.log" 2>&1 || { cat "$OUT/traffic.log"; exit 1; }
# the headline bench line with the fresh counter files, under --stats
cp "$OUT/pmc_latest.json" "$OUT/traffic_latest.json" /tmp/
step stats 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python bench.py --pmc-json /tmp/pmc_latest.json --traffic-json /tmp/traffic_latest.json --critical-path off ${BENCH_ARGS:-}
grep '^{' "$OUT/stats.log" > "$OUT/bench_stats.json" || true
python tools/trace_kernel_ms.py "$OUT/prof" --warmup 3 --steps ${STATS_STEPS:-96} --bench-json "$OUT/bench_stats.json" > "$OUT/kernel_ms_agreement.json" 2>&1
cat "$OUT/kernel_ms_agreement.json"
echo "session done"
