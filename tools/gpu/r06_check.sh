# round 6: GPU suite + smoke + default bench + 2-rank gloo rehearsal on the current tree
set -e
mkdir -p gpurun_out/r06a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r06a/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r06a/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r06a/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06a/smoke.log 2>&1 || { tail -20 gpurun_out/r06a/smoke.log; exit 1; }
tail -1 gpurun_out/r06a/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/r06a/bench_default.json 2> gpurun_out/r06a/bench_default.err
python -c "import json;d=json.load(open('gpurun_out/r06a/bench_default.json'));r=d['roofline'];print('default','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel'],r['launch_stats'],'mm',r['with_minmax_in']['ratio'])"
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/r06a/bench_gloo2.json 2> gpurun_out/r06a/bench_gloo2.err
python -c "import json;d=json.loads([l for l in open('gpurun_out/r06a/bench_gloo2.json') if l.startswith('{')][-1]);print('gloo2','%.4e'%d['value'],json.dumps(d['dist']['devices']), d['dist']['distinct_devices'])"
