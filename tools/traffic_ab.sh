#!/bin/bash
# HBM traffic (FETCH_SIZE / WRITE_SIZE PMC passes over the headline bench
# command) of variant libraries, then their interleaved throughput A/B.
#   LIBS="a b" SESSION=name bash tools/traffic_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
OUT=gpurun_out/${SESSION:-tab}
mkdir -p "$OUT"
V=schwarzschild-raytracer_amd/lib/variants
BENCH="bench.py --steps 8 --warmup 4 --cpu-baseline off --critical-path off --reference-loop off"
L=""
for n in $LIBS; do
  L="$L $V/libsr_$n.so"
  for c in FETCH_SIZE WRITE_SIZE; do
    SR_LIB=$V/libsr_$n.so timeout -k 10 180 rocprofv3 --kernel-trace --pmc $c -d "$OUT/$n-$c" -o run --output-format csv \
      -- python $BENCH > "$OUT/$n-$c.log" 2>&1 || { echo "$n $c rc=$?"; tail -5 "$OUT/$n-$c.log"; exit 1; }
  done
  python tools/traffic_json.py --frame "$OUT/$n-FETCH_SIZE" "$OUT/$n-WRITE_SIZE" --out "$OUT/traffic_$n.json" > "$OUT/traffic_$n.log" 2>&1 \
    || { cat "$OUT/traffic_$n.log"; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'MB/frame', round(d['hbm_bytes_per_frame']/1e6,1), 'write', round(d['write_bytes']/d['frames_per_launch']/1e6,1), 'fetch', round(d['fetch_bytes_raw']/d['frames_per_launch']/1e6,1))" "$OUT/traffic_$n.json" "$n"
done
timeout -k 10 500 python tools/ab_variants.py $L --throughput --rounds ${ROUNDS:-4} > "$OUT/ab_tp.log" 2>&1 || { tail -20 "$OUT/ab_tp.log"; exit 1; }
grep -E '"lib|median_ms_per_frame|identical' "$OUT/ab_tp.log"
echo "session done"
