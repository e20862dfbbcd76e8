#!/bin/bash
# Interleaved runs of the driver's headline command on one box, over
# libraries and/or option sets: LIBS="a b" (SR_LIB: lib/variants/libsr_<name>.so,
# "cur" = lib/libsr.so) x ARGSETS="opts1|opts2" (extra bench.py options, "-" for
# none), ROUNDS rounds:  LIBS="r5 cur" ROUNDS=3 SESSION=name bash tools/bench_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/${SESSION:-bench_ab}
mkdir -p "$OUT"
V=$PWD/schwarzschild-raytracer_amd/lib
IFS='|' read -r -a SETS <<< "${ARGSETS:--}"
for r in $(seq 1 ${ROUNDS:-3}); do
  for n in ${LIBS:-cur}; do
    for k in "${!SETS[@]}"; do
      a=${SETS[$k]}; [ "$a" = "-" ] && a=""
      lib=$V/variants/libsr_$n.so; [ "$n" = cur ] && lib=$V/libsr.so
      tag=${n}_a${k}_$r
      SR_LIB=$lib timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off ${BENCH_ARGS:-} $a \
        > "$OUT/$tag.log" 2>&1 || { tail -n 20 "$OUT/$tag.log"; exit 1; }
      grep '^{' "$OUT/$tag.log" > "$OUT/$tag.json"
      python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], (d['config'].get('single_frame') or {}).get('alone', {}).get('ms_per_frame'))" "$OUT/$tag.json" "$tag [$a]"
    done
  done
done
