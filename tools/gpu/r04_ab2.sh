# HISTORICAL (record of profiles/r04_experiments.json): the 8-wave / phase-locked / priority variants it
# compares were removed from the sources after the measurement (commit 83d898f); it no longer runs as written.
# wave-kernel priority A/B (libmzh.so = MLP phase at priority 1; prio1 = tree phases at priority 1;
# prio2 = no s_setprio), the cooperative tile's tree phase on 4 vs 8 waves, instruction mix at 65,536 roots
set -e
mkdir -p gpurun_out
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-tree --no-minmax-leg --steps 10 --warmup 2"
show() { python -c "import json;d=json.load(open('$1'));r=d['roofline'];print('$1',r['kernel'],'%.4f ms'%r['kernel_ms'],'frac %.4f'%r['frac'])"; }
for rep in 1 2; do
  for lib in libmzh libmzh_prio1 libmzh_prio2; do
    L=""; [ $lib != libmzh ] && L="MZH_LIB=$PWD/muzero-hanoi_amd/$lib.so"
    env $L $B > gpurun_out/ab_${lib}_c2_$rep.json 2> gpurun_out/ab2.err && show gpurun_out/ab_${lib}_c2_$rep.json
    env $L $B --config 2 --shard 0/2 > gpurun_out/ab_${lib}_s32k_$rep.json 2>> gpurun_out/ab2.err && show gpurun_out/ab_${lib}_s32k_$rep.json
  done
done
for cw in 4 8 4 8; do
  MZH_COOP_WAVES=$cw timeout -k 10 120 python bench.py --config 2 --shard 0/8 --no-cpu-baseline --no-minmax-leg --steps 10 > gpurun_out/ab_tree_cw$cw.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/ab_tree_cw$cw.json'));r=d['roofline'];t=r['tree'];print('cw$cw',r['kernel'],'%.4f ms'%r['kernel_ms'],'frac %.4f'%r['frac'],'tree',t['kernel'],'%.4f ms'%t['kernel_ms'])"
done
MZH_COOP_WAVES=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "full_size or sharded or caller_bounds or (coop and (deep or vs_oracle))" > gpurun_out/ab_cw8_tests.log 2>&1; tail -2 gpurun_out/ab_cw8_tests.log
bash tools/pmc_mix.sh "" c2 "mzh_wave_kernel<2, false" > /dev/null && cat gpurun_out/pmcmix_c2.json
