# wave-kernel A/B: stamps (diag build, skipped with NOSTAMP=1) + bench of libmzh.so and every
# libmzh_<tag>.so fast variant at the metric batch (65536 roots)
set -e
mkdir -p gpurun_out
if [ -z "$NOSTAMP" ]; then
  timeout -k 10 120 python tools/wave_probe.py > gpurun_out/wave_stamps.json 2>gpurun_out/wave_stamps.err
  cat gpurun_out/wave_stamps.json
fi
for lib in muzero-hanoi_amd/libmzh.so muzero-hanoi_amd/libmzh_[a-z]*.so; do
  case "$lib" in *diag*) continue;; esac
  tag=$(basename "$lib" .so)
  MZH_LIB=$PWD/$lib timeout -k 10 200 python bench.py --roots-per-gpu 65536 --steps 5 --warmup 2 --no-cpu-baseline --kernel wave > gpurun_out/ab_$tag.json 2>gpurun_out/ab_$tag.err
  python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print('$tag', '%.4e'%d['value'], '%.3f'%d['ms_per_step'], '%.4f'%d['roofline']['frac'])"
done
