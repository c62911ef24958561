# the two-workgroups-per-CU cooperative kernel (occ2): its parity tests, then same-box bench lines against
# the default kernel at the small per-GPU batches (configs[2]'s N=8 shard, configs[1]), interleaved rounds
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "occ2" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/occ2_tests.log 2>&1 || { tail -30 gpurun_out/occ2_tests.log; exit 1; }
tail -1 gpurun_out/occ2_tests.log
for r in 1 2 3; do
  for k in auto occ2; do
    for cfg in "--config 2 --shard 7/8" ${OCC2_CFG1:+"--config 1"}; do
      timeout -k 10 200 python bench.py $cfg --kernel $k --steps 20 --warmup 3 --no-cpu-baseline --no-tree --no-minmax-leg > gpurun_out/occ2_ab.json 2>>gpurun_out/occ2_ab.err
      python -c "import json;d=json.load(open('gpurun_out/occ2_ab.json'));r=d['roofline'];print('round $r', '$cfg', '$k', r['kernel'], '%.4f ms'%r['kernel_ms'], 'frac %.4f'%r['frac'])"
    done
  done
done
