# compare the three search kernels on mid-size batches (one bench line each)
set -e
mkdir -p gpurun_out
for cfg in "50 8192" "50 16384" "50 24576" "50 32768" "200 16384" "200 32768"; do
  set -- $cfg
  for k in coop wave16 wave; do
    timeout -k 10 200 python bench.py --sims $1 --roots-per-gpu $2 --steps 3 --warmup 1 --no-cpu-baseline --kernel $k > gpurun_out/kc.json 2>>gpurun_out/kc.err
    python -c "import json;d=json.load(open('gpurun_out/kc.json'));print('S=$1 B=$2 $k', '%.3e'%d['value'], 'frac %.3f'%d['roofline']['frac'])"
  done
done
