cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py -k cpp -x -v --timeout 300 --timeout-method thread > $OUT/pytest_cpp.log 2>&1; rc=$?; tail -3 $OUT/pytest_cpp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/cpp_driver_bench.py --rounds 3 > $OUT/cpp_vs_bench.jsonl 2> $OUT/cpp_vs_bench.err; rc=$?; tail -2 $OUT/cpp_vs_bench.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?; grep '^{' $OUT/bench.log > $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['config']['single_frame'], d['cpu_baseline']['sample'])"
timeout -k 10 400 python tools/split_sweep.py --split 0:16:1 64:16:1000 128:16:1000 256:16:800 512:16:600 64:4:1000 128:4:1000 256:4:800 --inflight 1 4 > $OUT/split_sweep.jsonl 2> $OUT/split_sweep.err; rc=$?; tail -3 $OUT/split_sweep.jsonl; [ $rc -eq 0 ] || exit $rc
