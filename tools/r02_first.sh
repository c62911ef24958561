# round-2 first GPU pass: parity suite, then bench lines at the BASELINE configs (each step time-limited)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for B in 65536 8192 4096; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --roots-per-gpu $B > gpurun_out/bench_$B.json 2>gpurun_out/bench_$B.err
  cat gpurun_out/bench_$B.json
done
