# parity suite, then bench lines for both search kernels: 8,192 / 4,096 roots (cooperative),
# 16,384 (wave16) and the default 65,536 (wave)
#   SKIP_TESTS=1 bash tools/iter_all.sh   -- timing only
set -e
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
fi
for B in 8192 4096 16384 65536; do
  timeout -k 10 120 python bench.py --roots-per-gpu $B --no-cpu-baseline > gpurun_out/bench_$B.json
  python -c "import json;d=json.load(open('gpurun_out/bench_$B.json'));r=d['roofline'];print($B,'%.4e'%d['value'],'%.4f'%r['frac'],r['kernel_ms'],'tree_ms',r['tree']['kernel_ms'])"
done
