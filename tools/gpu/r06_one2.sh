# latency kernel: parity of its tests, phase stamps, crossover probe, self-play drop-in
set -e
mkdir -p gpurun_out/r06d
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "one" > gpurun_out/r06d/one_tests.log 2>&1 || { tail -40 gpurun_out/r06d/one_tests.log; exit 1; }
tail -1 gpurun_out/r06d/one_tests.log
MZH_DIAG_LIB=muzero-hanoi_amd/libmzh_diag.so timeout -k 10 120 python tools/one_stamps.py > gpurun_out/r06d/stamps.json
python -c "import json;d=json.load(open('gpurun_out/r06d/stamps.json'));print(d['wave0_total'],d['sel_steps_per_sim'],d['ticks_per_sim']['wave0'])"
timeout -k 10 300 python tools/one_probe.py --out gpurun_out/r06d/one_probe.json > gpurun_out/r06d/one_probe.log 2>&1 || { tail -20 gpurun_out/r06d/one_probe.log; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/r06d/one_probe.json'))
for r in d['rows']: print(r['disks'],r['sims'],r['roots'],'one %.3f coop %.3f'%(r['one_ms'],r['coop_ms']),r['identical'])
print(d['run_mcts'])"
timeout -k 10 300 python tools/bench_selfplay.py --legs drop-in --out gpurun_out/r06d/selfplay.json > gpurun_out/r06d/selfplay.log 2>&1 || { tail -20 gpurun_out/r06d/selfplay.log; exit 1; }
tail -1 gpurun_out/r06d/selfplay.log
timeout -k 10 300 python tools/bench_env.py --out gpurun_out/r06d/env_bench.json > gpurun_out/r06d/env_bench.log 2>&1 || { tail -20 gpurun_out/r06d/env_bench.log; exit 1; }
cat gpurun_out/r06d/env_bench.log | grep leg
