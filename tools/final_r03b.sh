# round-end GPU pass (round 3, second session): as tools/final_r03.sh plus the 16,384 / 32,768-root shards (configs[2] at N=4 / N=2)
# configs[2] with the CPU baseline), configs[2]'s 8-GPU shard, a 2-rank gloo rehearsal, then rocprofv3
# stats + PMC at 65,536 / 8,192 / 4,096 roots with the traffic entries bench.py reads
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
rm -f gpurun_out/traffic_latest.json
TAG=c2 BENCH_ARGS="" bash tools/prof.sh
python tools/traffic.py gpurun_out c2 --traffic-json gpurun_out/traffic_latest.json > gpurun_out/traffic_c2.json
TAG=b8192 BENCH_ARGS="--roots-per-gpu 8192" bash tools/prof.sh
python tools/traffic.py gpurun_out b8192 --traffic-json gpurun_out/traffic_latest.json --roots-per-gpu 8192 > gpurun_out/traffic_b8192.json
TAG=c1 BENCH_ARGS="--config 1" bash tools/prof.sh
python tools/traffic.py gpurun_out c1 --traffic-json gpurun_out/traffic_latest.json --config 1 > gpurun_out/traffic_c1.json
cp gpurun_out/traffic_latest.json profiles/traffic_latest.json
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
cat gpurun_out/bench_default.json
for C in 1 3 4; do
  timeout -k 10 200 python bench.py --config $C --no-cpu-baseline > gpurun_out/bench_c$C.json 2> gpurun_out/bench_c$C.err
  python -c "import json;d=json.load(open('gpurun_out/bench_c$C.json'));r=d['roofline'];print('c$C','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel_ms'],'traffic',r['traffic'])"
done
timeout -k 10 120 python bench.py --roots-per-gpu 8192 --no-cpu-baseline > gpurun_out/bench_8192.json 2> gpurun_out/bench_8192.err
python -c "import json;d=json.load(open('gpurun_out/bench_8192.json'));r=d['roofline'];print('8192','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel_ms'],'traffic',r['traffic'])"
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
tail -c 300 gpurun_out/bench_gloo2.json
for B in 16384 32768; do
  timeout -k 10 120 python bench.py --roots-per-gpu $B --no-cpu-baseline > gpurun_out/bench_$B.json 2> gpurun_out/bench_$B.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$B.json'));r=d['roofline'];print('$B','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel_ms'])"
done
