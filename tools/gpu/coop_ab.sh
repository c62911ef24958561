# a cooperative-kernel change: the GPU suite on it, then interleaved A/B rounds against the base build
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/coop_tests.log 2>&1
rc=$?; [ -n "$SKIP_TESTS" ] && rc=0
echo "tests rc=$rc"; tail -3 gpurun_out/coop_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
ROUNDS=${ROUNDS:-3} bash tools/ab_libs.sh muzero-hanoi_amd/libmzh_base.so muzero-hanoi_amd/libmzh.so 2>&1 | grep -v amdgpu.ids
