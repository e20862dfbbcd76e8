#!/bin/bash
# r4 s34: the C++ node driver at the new one-GPU default shape (16 x 2)
# against bench.py, interleaved, 96 frames; its GPU test
cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r4s34; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py -m gpu -k cpp -x -q --timeout 300 --timeout-method thread > $OUT/pytest_cpp.log 2>&1; rc=$?; tail -2 $OUT/pytest_cpp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/cpp_driver_bench.py --rounds 3 --frames 96 > $OUT/cpp_vs_bench.jsonl 2> $OUT/cpp_vs_bench.err; rc=$?; tail -1 $OUT/cpp_vs_bench.jsonl; [ $rc -eq 0 ] || { tail -5 $OUT/cpp_vs_bench.err; exit $rc; }
