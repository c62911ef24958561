# BASELINE.json configs on one GPU (auto kernel choice), one bench line each
set -e
mkdir -p gpurun_out
for cfg in "4 50 4096" "4 50 8192" "4 50 16384" "4 50 32768" "4 50 65536" "4 50 131072" "4 200 16384" "7 100 32768" "3 25 65536"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --disks $1 --sims $2 --roots-per-gpu $3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/sweep_$1_$2_$3.json 2>>gpurun_out/sweep.err
  python -c "import json;d=json.load(open('gpurun_out/sweep_$1_$2_$3.json'));r=d['roofline'];print('N=$1 S=$2 B=$3', '%.3e'%d['value'], '%.3f ms'%d['ms_per_step'], 'frac %.3f'%r['frac'], r['kernel'])"
done
