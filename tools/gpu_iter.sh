# one GPU iteration: parity tests -> stamps (A/B variants) -> phase probe -> short bench (each step time-limited)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps.json 2>/dev/null
bash tools/ab_variants.sh
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err
cat gpurun_out/bench.json
