# round 6: the latency kernel -- parity tests of it first, then the full GPU suite, the crossover probe, self-play
set -e
mkdir -p gpurun_out/r06b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "one" > gpurun_out/r06b/one_tests.log 2>&1 || { tail -40 gpurun_out/r06b/one_tests.log; exit 1; }
tail -1 gpurun_out/r06b/one_tests.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06b/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r06b/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06b/gpu_tests.log
timeout -k 10 300 python tools/one_probe.py --out gpurun_out/r06b/one_probe.json > gpurun_out/r06b/one_probe.log 2>&1 || { tail -20 gpurun_out/r06b/one_probe.log; exit 1; }
tail -3 gpurun_out/r06b/one_probe.log
timeout -k 10 300 python tools/bench_selfplay.py --legs batched,drop-in --out gpurun_out/r06b/selfplay.json > gpurun_out/r06b/selfplay.log 2>&1 || { tail -20 gpurun_out/r06b/selfplay.log; exit 1; }
tail -4 gpurun_out/r06b/selfplay.log
