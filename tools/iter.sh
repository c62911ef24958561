set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
ROUNDS=2 bash tools/ab_libs.sh ${LIBS:-muzero-hanoi_amd/libmzh_base.so muzero-hanoi_amd/libmzh.so}
timeout -k 10 120 python tools/stamp_probe.py 8192 > gpurun_out/stamps_8192.json
