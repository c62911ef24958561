# A/B of library builds at small batches: bash tools/ab_libs.sh LIB [LIB ...] (paths relative to the repo),
# ROOTS (default "8192 4096"), ROUNDS interleaved rounds; coop kernel forced
set -e
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-1}); do
for B in ${ROOTS:-8192 4096}; do
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  MZH_LIB=$PWD/$lib timeout -k 10 120 python bench.py --roots-per-gpu $B --no-cpu-baseline --no-tree --kernel ${KERNEL:-coop} > gpurun_out/ab_${tag}_$B.json
  python -c "import json;d=json.load(open('gpurun_out/ab_${tag}_$B.json'));print('r$r', $B, '$tag', '%.4e'%d['value'],'%.4f'%d['roofline']['frac'],'%.4f'%d['roofline']['kernel_ms'])"
done; done; done
