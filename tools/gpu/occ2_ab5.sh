set -e
mkdir -p gpurun_out
for r in 1 2 3 4 5; do
  for k in auto occ2; do
    timeout -k 10 200 python bench.py --config 2 --shard 7/8 --kernel $k --steps 30 --warmup 3 --no-cpu-baseline --no-tree --no-minmax-leg > gpurun_out/occ2_ab.json 2>>gpurun_out/occ2_ab.err
    python -c "import json;d=json.load(open('gpurun_out/occ2_ab.json'));r=d['roofline'];print('round $r', '$k', r['kernel'], '%.4f ms'%r['kernel_ms'], 'frac %.4f'%r['frac'])"
  done
done
