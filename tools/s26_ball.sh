cd "${GRAFT_REPO_ROOT}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/s26; mkdir -p $OUT
V=$PWD/schwarzschild-raytracer_amd/lib/variants
SR_LIB=$V/libsr_ball.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $OUT/pytest_ball.log 2>&1; rc=$?
tail -15 $OUT/pytest_ball.log
[[ $rc == 0 || $rc == 1 ]] || exit $rc
PYTEST=0 LIBS="head ball" SESSION=s26 ROUNDS=3 bash tools/ab_session.sh
