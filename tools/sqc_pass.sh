cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=8
O=gpurun_out/s36; mkdir -p $O
timeout -k 5 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQC_[A-Z_0-9]*" $O/counters.txt | sort -u > $O/sqc_names.txt; cat $O/sqc_names.txt | head -40
if grep -q "^SQC_DCACHE_MISSES$" $O/sqc_names.txt && grep -q "^SQC_DCACHE_HITS$" $O/sqc_names.txt; then
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES -d $O/p1 -o run --output-format csv -- python bench.py --steps 8 --warmup 4 --cpu-baseline off --critical-path off --reference-loop off > $O/p1.log 2>&1
  echo "p1 rc=$?"
fi
