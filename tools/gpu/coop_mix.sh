# PMC instruction mix + wait split of the cooperative kernel at 8,192 and 4,096 roots on the current build
# (tools/pmc_mix.sh), for comparison with profiles/r05_pmcmix.json (the build before round 5's second session)
set -e
mkdir -p gpurun_out
bash tools/pmc_mix.sh "--no-tree --config 2 --shard 7/8" b8192 "search_kernel<32, false" > gpurun_out/mix_b8192.log 2>&1 || { tail -20 gpurun_out/mix_b8192.log; exit 1; }
bash tools/pmc_mix.sh "--no-tree --config 1" c1 "search_kernel<16, false" > gpurun_out/mix_c1.log 2>&1 || { tail -20 gpurun_out/mix_c1.log; exit 1; }
echo done
