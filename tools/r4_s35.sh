#!/bin/bash
# r4 s35: the round-end checks at the final tree: smoke(), the driver's bench
# command, and its rocprofv3 --kernel-trace --stats summary
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s35; mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver_cmd.log 2>&1; rc=$?; grep '^{' $OUT/bench_driver_cmd.log > $OUT/bench_driver_cmd.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench_driver_cmd.json')); print(d['value'], d['ms_per_step'], d['config']['frames_per_launch'], d['config']['launches_in_flight'], d['roofline'].get('frac'), d['parity']['frame_sha_match'], d['cpu_baseline']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > $OUT/prof.log 2>&1; rc=$?; [ $rc -eq 0 ] || { tail -5 $OUT/prof.log; exit $rc; }
find $OUT/prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
head -4 $OUT/kernel_stats.csv | cut -c1-200
