# one GPU iteration: parity tests -> stamps -> phase probe -> short bench (each step time-limited)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps.json 2>/dev/null
timeout -k 10 200 python tools/phase_probe.py > gpurun_out/probe.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.json 2>gpurun_out/bench.err
cat gpurun_out/probe.json; echo; cat gpurun_out/bench.json
echo
MZH_ROWS=16 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_R16.json 2>/dev/null && cat gpurun_out/bench_R16.json | python -c "import json,sys; d=json.load(sys.stdin); print('R16', d['value'], d['roofline']['kernel_ms'])"
