cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/s6 && export TMPDIR=/tmp
V=schwarzschild-raytracer_amd/lib/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "two_rays" -v --timeout 120 --timeout-method thread --tb=short > gpurun_out/s6/pytest_pair.log 2>&1; rc=$?
grep -E "^E |differs|Error|PASS|FAIL" gpurun_out/s6/pytest_pair.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_variants.py $V/libsr_single.so $V/libsr_pair5.so $V/libsr_pair4.so $V/libsr_base.so --throughput --rounds 4 > gpurun_out/s6/ab_tp.log 2>&1 || exit $?
tail -40 gpurun_out/s6/ab_tp.log
timeout -k 10 300 python tools/ab_variants.py $V/libsr_single.so $V/libsr_pair5.so $V/libsr_pair4.so --rounds 4 > gpurun_out/s6/ab_single.log 2>&1 || exit $?
tail -30 gpurun_out/s6/ab_single.log
