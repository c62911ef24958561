set -e
mkdir -p gpurun_out
for r in 1 2; do
for T in 32 16; do
  timeout -k 10 120 python bench.py --roots-per-gpu 8192 --no-cpu-baseline --kernel coop --tile $T > gpurun_out/occ_$T.json
  python -c "import json;d=json.load(open('gpurun_out/occ_$T.json'));print('r$r tile $T', '%.4e'%d['value'],'%.4f'%d['roofline']['frac'],'%.4f'%d['roofline']['kernel_ms'], 'tree', '%.4f'%d['roofline']['tree']['kernel_ms'])"
done; done
