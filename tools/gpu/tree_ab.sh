# replay (tree-only) instantiation timing per kernel: bench lines with the live tree measurement
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for B in 65536 16384; do for k in wave wave16; do
  timeout -k 10 120 python bench.py --roots-per-gpu $B --no-cpu-baseline --kernel $k --steps 10 > gpurun_out/tab_${k}_$B.json || exit $?
  python -c "import json;d=json.load(open('gpurun_out/tab_${k}_$B.json'));r=d['roofline'];t=r['tree'];print($B,'$k','fused %.4f'%r['kernel_ms'],'tree %.4f ms frac %.3f'%(t['kernel_ms'],t['frac']))"
done; done
