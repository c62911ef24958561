# HISTORICAL (record of profiles/r04_experiments.json): the 8-wave / phase-locked / priority variants it
# compares were removed from the sources after the measurement (commit 83d898f); it no longer runs as written.
# instruction mix of the wave kernel at configs[2] on one GPU (65,536 roots, NT=2) and its 16,384-root shard (NT=1)
set -e
bash tools/pmc_mix.sh "" c2 "mzh_wave_kernel<2, false" > /dev/null
bash tools/pmc_mix.sh "--config 2 --shard 0/4" s16k "mzh_wave_kernel<1, false" > /dev/null
cat gpurun_out/pmcmix_c2.json gpurun_out/pmcmix_s16k.json
# the cooperative 32-root tile's tree phase (replay instantiation: no MLP) on 4 vs 8 waves
for cw in 4 8 4 8; do
  MZH_COOP_WAVES=$cw timeout -k 10 120 python bench.py --config 2 --shard 0/8 --no-cpu-baseline --no-minmax-leg --steps 3 > gpurun_out/ab_tree_cw$cw.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/ab_tree_cw$cw.json'));t=d['roofline']['tree'];print('cw$cw',t['kernel'],'%.4f ms'%t['kernel_ms'])"
done
