# bin 32 of the 33-bin heads by vector chains (two MFMA tiles instead of three): GPU tests on the new build,
# then A/B against the previous build (libmzh_base.so) on every kernel's workload
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-tree --no-minmax-leg --steps 10 --warmup 2"
show() { python -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$1','%.4f ms'%r['kernel_ms'],'frac %.4f'%r['frac'])"; }
for rep in 1 2; do
  for lib in libmzh_base libmzh; do
    L=""; [ $lib != libmzh ] && L="MZH_LIB=$PWD/muzero-hanoi_amd/$lib.so"
    for w in "c2:" "s32k:--config 2 --shard 0/2" "s8k:--config 2 --shard 0/8" "c1:--config 1" "c4:--config 4 --steps 4"; do
      T=${w%%:*}; A=${w#*:}
      env $L $B $A > gpurun_out/ab3_${lib}_${T}_$rep.json 2>> gpurun_out/ab3.err && show gpurun_out/ab3_${lib}_${T}_$rep.json
    done
  done
done
