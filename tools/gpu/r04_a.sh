# round 4, first GPU pass: the plan-query build's GPU tests + smoke, the default bench line, and the
# configs[4] 8-GPU shard (rank 0 of 8, 32,768 roots at N=7, S=100) benched and profiled
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --cpu-baseline-seconds 6 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('c2','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel'],r['kernel_ms'],'mm',r['with_minmax_in'])"
rm -f gpurun_out/traffic_latest.json
TAG=c4s8 BENCH_ARGS="--config 4 --shard 0/8" bash tools/prof.sh
python tools/traffic.py gpurun_out c4s8 --traffic-json gpurun_out/traffic_latest.json > gpurun_out/traffic_c4s8.json
timeout -k 10 200 python bench.py --config 4 --shard 0/8 --no-cpu-baseline > gpurun_out/bench_c4s8.json 2> gpurun_out/bench_c4s8.err
python -c "import json;d=json.load(open('gpurun_out/bench_c4s8.json'));r=d['roofline'];print('c4s8','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel'],r['kernel_ms'],'traffic',r['traffic'])"
