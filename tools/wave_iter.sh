# GPU iteration for the wave kernel: new parity tests, then coop vs wave bench at the metric batch
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "wave or deep" > gpurun_out/wave_tests.log 2>&1 || { tail -40 gpurun_out/wave_tests.log; exit 1; }
tail -2 gpurun_out/wave_tests.log
for k in coop wave; do
  timeout -k 10 200 python bench.py --roots-per-gpu 65536 --steps 5 --warmup 2 --no-cpu-baseline --kernel $k > gpurun_out/bench_$k.json 2>gpurun_out/bench_$k.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$k.json'));print('$k', '%.3e'%d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
