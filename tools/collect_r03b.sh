# copy a round-end GPU pass (tools/final_r03.sh) from gpurun_out/ into profiles/ under a prefix
#   bash tools/collect_r03.sh r03f
set -e
P=${1:-r03}
for t in c2 b8192 c1; do
  ks=$(ls -t gpurun_out/prof_${t}_trace/*/*_kernel_stats.csv | head -1)
  cp "$ks" profiles/${P}_${t}_kernel_stats.csv
  cp gpurun_out/traffic_${t}.json profiles/${P}_${t}_prof_summary.json
done
for b in default c1 c3 c4 8192 16384 32768 gloo2; do cp gpurun_out/bench_$b.json profiles/${P}_bench_$b.json; done
cp gpurun_out/traffic_latest.json profiles/traffic_latest.json
tail -1 gpurun_out/gpu_tests.log > profiles/${P}_gpu_tests.txt
tail -1 gpurun_out/smoke.log >> profiles/${P}_gpu_tests.txt
