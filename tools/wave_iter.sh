# wave-kernel iteration: parity suite, then A/B of libmzh_prev.so vs libmzh.so at the wave (65,536)
# and wave16 (16,384 / 32,768) batches, two interleaved rounds (each step time-limited)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
ROUNDS=2 KERNEL=wave ROOTS=65536 bash tools/ab_libs.sh muzero-hanoi_amd/libmzh_prev.so muzero-hanoi_amd/libmzh.so
ROUNDS=1 KERNEL=wave16 ROOTS="16384 32768" bash tools/ab_libs.sh muzero-hanoi_amd/libmzh_prev.so muzero-hanoi_amd/libmzh.so
