# generic same-box A/B of library builds: bash tools/gpu/ab.sh "libmzh libmzh_x ..." "TAG:BENCH_ARGS" ...
# two interleaved rounds; HIP-event kernel ms from bench.py (no CPU baseline, no tree leg, no minmax leg)
set -e
mkdir -p gpurun_out
LIBS=$1; shift
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-tree --no-minmax-leg --steps 10 --warmup 2"
for rep in ${AB_REPS:-1 2}; do
  for lib in $LIBS; do
    L=""; [ $lib != libmzh ] && L="MZH_LIB=$PWD/muzero-hanoi_amd/$lib.so"
    for w in "$@"; do
      T=${w%%:*}; A=${w#*:}
      env $L $B $A > gpurun_out/ab_${lib}_${T}_$rep.json 2>> gpurun_out/ab.err
      python -c "import json;d=json.load(open('gpurun_out/ab_${lib}_${T}_$rep.json'));r=d['roofline'];print('$lib $T $rep','%.4f ms'%r['kernel_ms'],'frac %.4f'%r['frac'])"
    done
  done
done
