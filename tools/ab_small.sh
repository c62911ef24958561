set -e
mkdir -p gpurun_out
for lib in muzero-hanoi_amd/libmzh.so muzero-hanoi_amd/libmzh_w8.so; do
  tag=$(basename $lib .so)
  for cfg in "1 25 3" "16 25 3" "4096 50 4"; do
    set -- $cfg
    MZH_LIB=$PWD/$lib timeout -k 10 120 python bench.py --roots-per-gpu $1 --sims $2 --disks $3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abs_${tag}_$1.json 2>gpurun_out/abs_${tag}_$1.err
    python -c "import json;d=json.load(open('gpurun_out/abs_${tag}_$1.json'));print('$tag B=$1', '%.4e'%d['value'], 'kern_ms %.4f'%d['roofline']['kernel_ms'])"
  done
  MZH_LIB=$PWD/$lib timeout -k 10 120 python tools/bench_selfplay.py --legs drop-in --dropin-seconds 8 > gpurun_out/abs_${tag}_sp.json 2>gpurun_out/abs_${tag}_sp.err
  echo "$tag selfplay $(tail -c 600 gpurun_out/abs_${tag}_sp.json)"
done
