# the two-workgroups-per-CU cooperative kernel (occ2) against the default 32-root tile, same box, interleaved
# rounds at configs[2]'s N=8 shard (OCC2_CFG1=1: configs[1] too; OCC2_ROUNDS: rounds, default 3; OCC2_TESTS=1:
# its parity tests first)
set -e
mkdir -p gpurun_out
if [ -n "$OCC2_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "occ2" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/occ2_tests.log 2>&1 || { tail -30 gpurun_out/occ2_tests.log; exit 1; }
  tail -1 gpurun_out/occ2_tests.log
fi
for r in $(seq 1 ${OCC2_ROUNDS:-3}); do
  for k in auto occ2; do
    for cfg in "--config 2 --shard 7/8" ${OCC2_CFG1:+"--config 1"}; do
      timeout -k 10 200 python bench.py $cfg --kernel $k --steps 30 --warmup 3 --no-cpu-baseline --no-tree --no-minmax-leg > gpurun_out/occ2_ab.json 2>>gpurun_out/occ2_ab.err
      python -c "import json;d=json.load(open('gpurun_out/occ2_ab.json'));r=d['roofline'];print('round $r', '$cfg', '$k', r['kernel'], '%.4f ms'%r['kernel_ms'], 'frac %.4f'%r['frac'])"
    done
  done
done
