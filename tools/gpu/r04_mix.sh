# instruction mix of the wave kernel at configs[2] on one GPU (65,536 roots, NT=2) and its 16,384-root shard (NT=1)
set -e
bash tools/pmc_mix.sh "" c2 "mzh_wave_kernel<2, false" > /dev/null
bash tools/pmc_mix.sh "--config 2 --shard 0/4" s16k "mzh_wave_kernel<1, false" > /dev/null
cat gpurun_out/pmcmix_c2.json gpurun_out/pmcmix_s16k.json
