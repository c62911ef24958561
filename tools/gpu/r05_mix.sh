# round 5: the memory probe (loaded latency / random-line bandwidth by footprint and concurrency), then the
# PMC instruction mix + wait split of the tree-only (replay) kernel at 65,536 roots and of the two 8,192-root
# forms (32-root tile; two 16-root workgroups per CU)
set -e
mkdir -p gpurun_out
timeout -k 10 180 ./tools/micro/tree_mem_probe > gpurun_out/tree_mem_probe.json
bash tools/pmc_mix.sh "" c2tree "_kernel<2, true" > gpurun_out/mix_c2tree.log 2>&1 || { tail -20 gpurun_out/mix_c2tree.log; exit 1; }
bash tools/pmc_mix.sh "--no-tree --config 2 --shard 7/8" b8192 "search_kernel<32, false" > gpurun_out/mix_b8192.log 2>&1 || { tail -20 gpurun_out/mix_b8192.log; exit 1; }
bash tools/pmc_mix.sh "--no-tree --config 2 --shard 7/8 --kernel occ2" b8192occ2 "occ2_kernel<" > gpurun_out/mix_b8192occ2.log 2>&1 || { tail -20 gpurun_out/mix_b8192occ2.log; exit 1; }
echo done
