# full GPU check: parity suite, rocprof stats + PMC at the bench batch and at 8,192 / 4,096 roots, bench line
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
TAG=c2 BENCH_ARGS="" bash tools/prof.sh
TAG=b8192 BENCH_ARGS="--roots-per-gpu 8192" bash tools/prof.sh
TAG=c1 BENCH_ARGS="--config 1" bash tools/prof.sh
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
cat gpurun_out/bench_default.json
