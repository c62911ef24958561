# A/B of cooperative-kernel variant builds at 4,096 / 8,192 roots, then their search parity tests
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-3} ROOTS="${ROOTS:-4096}" bash tools/ab_libs.sh $LIBS 2>&1 | grep -v amdgpu.ids || exit $?
for lib in $TESTLIBS; do
  MZH_LIB=$PWD/$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "coop or baseline or sharded or large_batch" > gpurun_out/ab_tests_$(basename $lib .so).log 2>&1
  rc=$?; echo "$lib tests rc=$rc $(tail -1 gpurun_out/ab_tests_$(basename $lib .so).log)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
