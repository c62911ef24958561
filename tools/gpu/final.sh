# final pass of a round: GPU tests + smoke on the final build, the driver's default bench command (with
# the CPU baseline), a 2-rank gloo rehearsal of the N>1 bench path on one GPU
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
python -c "import json;d=json.load(open('gpurun_out/bench_default.json'));r=d['roofline'];print('default','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel'],'cpu',d['cpu_baseline']['value'],'tree',r['tree']['frac'],'predraw_ms',d['predraw']['ms'])"
# N > 1 as the driver may start it: bench.py --gpus 2 with no launcher starts its own 2 ranks (gloo lets them share the one GPU)
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
python -c "import json;d=json.loads([l for l in open('gpurun_out/bench_gloo2.json') if l.startswith('{')][-1]);print('gloo2','%.4e'%d['value'],json.dumps(d['dist']))"  # gloo prints its connection lines on stdout
