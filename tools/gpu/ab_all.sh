# GPU suite on the working build, then interleaved A/B vs libmzh_base.so at the bench's batch sizes (auto kernel)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_all_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/ab_all_tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
KERNEL=auto ROUNDS=${ROUNDS:-2} ROOTS="${ROOTS:-65536 16384 8192 4096}" bash tools/ab_libs.sh muzero-hanoi_amd/libmzh_base.so muzero-hanoi_amd/libmzh.so 2>&1 | grep -v amdgpu.ids
