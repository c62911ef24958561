# A/B of search kernels on one library: bash tools/kernel_ab.sh ; ROOTS (default "16384 32768 65536"),
# KERNELS (default "wave16 wave"), ROUNDS interleaved rounds, SIMS/DISKS optional
set -e
mkdir -p gpurun_out
for r in $(seq 1 ${ROUNDS:-1}); do
for B in ${ROOTS:-16384 32768 65536}; do
for k in ${KERNELS:-wave16 wave}; do
  timeout -k 10 120 python bench.py --roots-per-gpu $B --no-cpu-baseline --no-tree --kernel $k --steps ${STEPS:-10} \
    ${SIMS:+--sims $SIMS} ${DISKS:+--disks $DISKS} > gpurun_out/kab_${k}_$B.json
  python -c "import json;d=json.load(open('gpurun_out/kab_${k}_$B.json'));print('r$r', $B, '$k', '%.4e'%d['value'],'%.4f'%d['roofline']['frac'],'%.4f'%d['roofline']['kernel_ms'])"
done; done; done
