# coop-kernel iteration: parity suite, phase stamps and bench lines at 8,192 / 4,096 roots (each step time-limited)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for B in 8192 4096; do
  timeout -k 10 120 python tools/stamp_probe.py $B > gpurun_out/stamps_$B.json
  timeout -k 10 120 python bench.py --roots-per-gpu $B --no-cpu-baseline --no-tree > gpurun_out/bench_$B.json
  python -c "import json;d=json.load(open('gpurun_out/bench_$B.json'));print($B,'%.4e'%d['value'],'%.4f'%d['roofline']['frac'],d['roofline']['kernel_ms'])"
done
