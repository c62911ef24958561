# wave-kernel A/B: stamps (diag build, skipped with NOSTAMP=1) + bench of libmzh.so and every
# libmzh_<tag>.so fast variant at the metric batch (65536 roots), ROUNDS interleaved rounds
set -e
mkdir -p gpurun_out
if [ -z "$NOSTAMP" ]; then
  for dl in muzero-hanoi_amd/libmzh_diag*.so; do
    t=$(basename $dl .so)
    MZH_DIAG_LIB=$PWD/$dl timeout -k 10 120 python tools/wave_probe.py > gpurun_out/stamps_$t.json 2>gpurun_out/stamps_$t.err
    echo "$t $(cat gpurun_out/stamps_$t.json)"
  done
fi
for r in $(seq 1 ${ROUNDS:-1}); do
for lib in muzero-hanoi_amd/libmzh.so muzero-hanoi_amd/libmzh_[a-z]*.so; do
  case "$lib" in *diag*) continue;; esac
  tag=$(basename "$lib" .so)
  MZH_LIB=$PWD/$lib timeout -k 10 200 python bench.py --roots-per-gpu ${ROOTS:-65536} --steps 5 --warmup 2 --no-cpu-baseline --kernel wave > gpurun_out/ab_$tag.json 2>gpurun_out/ab_$tag.err
  python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print('r$r $tag', '%.4e'%d['value'], '%.3f'%d['ms_per_step'], '%.4f'%d['roofline']['frac'])"
done
done
