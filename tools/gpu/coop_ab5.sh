# parity (all GPU tests) on the working build, then A/B vs libmzh_base.so at 4,096 / 8,192 roots
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab5_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/ab5_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
ROUNDS=${ROUNDS:-3} ROOTS="${ROOTS:-4096 8192}" bash tools/ab_libs.sh muzero-hanoi_amd/libmzh_base.so muzero-hanoi_amd/libmzh.so 2>&1 | grep -v amdgpu.ids
