# cooperative kernel: bin 32 of the 33-bin heads on the idle fourth wave of the last MLP phase
# (bin-32 weights staged in LDS; R = 16 splits each row's chains over the half-waves)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-tree --no-minmax-leg --steps 10 --warmup 2"
show() { python -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$1','%.4f ms'%r['kernel_ms'],'frac %.4f'%r['frac'])"; }
for rep in 1 2; do
  for lib in libmzh_base libmzh; do
    L=""; [ $lib != libmzh ] && L="MZH_LIB=$PWD/muzero-hanoi_amd/$lib.so"
    for w in "s8k:--config 2 --shard 0/8" "c1:--config 1" "c1s2:--config 1 --shard 0/2" "c3s2:--config 3 --shard 0/2" "c2:"; do
      T=${w%%:*}; A=${w#*:}
      env $L $B $A > gpurun_out/ab5_${lib}_${T}_$rep.json 2>> gpurun_out/ab5.err && show gpurun_out/ab5_${lib}_${T}_$rep.json
    done
  done
done
