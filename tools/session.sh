#!/bin/bash
# One parameterised GPU-box session (replaces round 4's one-off r4_s*.sh
# scripts): the steps named in STEPS run in order, each under its own time
# limit; the first failure ends the session (no GPU step after a fault,
# abort or time limit).
#
#   STEPS="pytest smoke bench rocstats" SESSION=r5s1 bash tools/session.sh
#
# Steps (variant libraries are schwarzschild-raytracer_amd/lib/variants/libsr_<name>.so,
# built by tools/build_variant.sh):
#   pytest      GPU tests (TEST=<variant>: on that library via SR_LIB; PYTEST_ARGS)
#   smoke       __graft_entry__.smoke()
#   bench       the driver's headline command (BENCH_ARGS: extra bench.py options)
#   rocstats    rocprofv3 --kernel-trace --stats of the driver's headline command
#   ab          interleaved throughput and single-frame A/B of LIBS="a b"
#   stats       SR_STATS event counters of STATS="a b" (tools/stats_frame.py; STATS_ARGS)
#   prof        SR_PROF section cycles of PROF="a b" (tools/prof_waves.py; PROF_ARGS)
#   pmc         PMC passes (PASSES, one rocprofv3 run each) of PMC="a b" (tools/prof_frame.py)
#   traffic     FETCH_SIZE / WRITE_SIZE of the headline command for TRAFFIC="a b"
#   roofline    tools/roofline_session.sh (SESSION/BENCH_ARGS passed through)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${SESSION:-session}
mkdir -p "$OUT"
V=${SR_VARIANTS:-$PWD/schwarzschild-raytracer_amd/lib/variants}  # lib/variants stays out of the GPU push (.gpurunignore): a session copies what it needs to lib/ab
DRIVER="bench.py --gpus 1 --steps 20 --warmup 5"

step() {  # name timeout cmd... : logs to $OUT/name.log, stops the session on failure
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  [ $rc -eq 0 ] || { tail -n 25 "$OUT/$name.log"; exit $rc; }
}

for S in ${STEPS:-pytest smoke bench}; do
  case $S in
  pytest)
    if [ -n "$TEST" ]; then export SR_LIB=$V/libsr_$TEST.so; fi
    step pytest 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
    unset SR_LIB
    tail -n 3 "$OUT/pytest.log" ;;
  smoke)
    step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
    tail -n 1 "$OUT/smoke.log" ;;
  bench)
    step bench 400 python $DRIVER ${BENCH_ARGS:-}
    grep '^{' "$OUT/bench.log" > "$OUT/bench.json"
    python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
rf = d.get("roofline") or {}
sf = (d["config"].get("single_frame") or {}).get("alone") or {}
print("value", d["value"], "ms", d["ms_per_step"], "frac", rf.get("frac"), "parity", (d.get("parity") or {}).get("frame_sha_match"),
      "alone_ms", sf.get("ms_per_frame"), "band_ms", (rf.get("critical_path") or {}).get("band_ms"),
      "cpu", (d.get("cpu_baseline") or {}).get("value"))
PY
    ;;
  rocstats)
    # the queue count scoped to this step (a temporary assignment on the
    # function call), so later steps keep the box default
    GPU_MAX_HW_QUEUES=8 step rocstats 500 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python $DRIVER --cpu-baseline off ${BENCH_ARGS:-}
    find "$OUT/prof" -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} "$OUT/kernel_stats.csv"
    grep '^{' "$OUT/rocstats.log" > "$OUT/rocstats_bench.json" || true
    head -4 "$OUT/kernel_stats.csv" | cut -c1-200 ;;
  ab)
    L=""; for n in $LIBS; do L="$L $V/libsr_$n.so"; done
    step ab_tp 600 python tools/ab_variants.py $L --throughput --rounds ${ROUNDS:-4} ${AB_ARGS:-}
    grep -E '"lib|median_ms_per_frame|identical' "$OUT/ab_tp.log"
    step ab_single 400 python tools/ab_variants.py $L --rounds ${ROUNDS:-4} ${AB_ARGS:-}
    grep -E '"lib|median_ms"|identical' "$OUT/ab_single.log" ;;
  stats)
    for n in $STATS; do
      step "stats_$n" 240 python tools/stats_frame.py $V/libsr_$n.so ${STATS_ARGS:-}
      python -c "import json,sys; t=open(sys.argv[1]).read(); d=json.loads(t[t.index('{'):]); print(sys.argv[2], {k: d[k] for k in ('events', 'wave_steps', 'event_frac') if k in d}, [d.get('slot%d_spent' % j) for j in range(9)])" "$OUT/stats_$n.log" "$n"
    done ;;
  prof)
    for n in $PROF; do step "prof_$n" 240 python tools/prof_waves.py $V/libsr_$n.so ${PROF_ARGS:-}; done ;;
  pmc)
    PASSES=${PASSES:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"}
    for v in $PMC; do
      i=0
      while read -r line; do
        [ -z "$line" ] && continue
        i=$((i + 1))
        SR_LIB=$V/libsr_$v.so step "pmc_${v}_p$i" 120 rocprofv3 --kernel-trace --pmc $line -d "$OUT/pmc_$v/p$i" -o run --output-format csv -- python tools/prof_frame.py --frames 2 ${PROF_ARGS:-}
      done <<< "$PASSES"
      python tools/pmc_summary.py "$OUT/pmc_$v"
    done ;;
  traffic)
    B="bench.py --steps 8 --warmup 4 --cpu-baseline off --critical-path off --reference-loop off --single-frame off"
    for n in $TRAFFIC; do
      for c in FETCH_SIZE WRITE_SIZE; do
        GPU_MAX_HW_QUEUES=8 SR_LIB=$V/libsr_$n.so step "traffic_${n}_$c" 180 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$n-$c" -o run --output-format csv -- python $B
      done
      python tools/traffic_json.py --frame "$OUT/$n-FETCH_SIZE" "$OUT/$n-WRITE_SIZE" --out "$OUT/traffic_$n.json" > "$OUT/traffic_$n.log" 2>&1 \
        || { cat "$OUT/traffic_$n.log"; exit 1; }
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'MB/frame', round(d['hbm_bytes_per_frame']/1e6,1))" "$OUT/traffic_$n.json" "$n"
    done ;;
  roofline)
    SESSION=${SESSION:-session}/roof bash tools/roofline_session.sh || exit $? ;;
  *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "session done"
