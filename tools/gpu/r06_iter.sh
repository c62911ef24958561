# latency-kernel iteration: parity of its tests, phase stamps (every wave), crossover probe, self-play drop-in
#   OUT=gpurun_out/<dir> bash tools/gpu/r06_iter.sh
set -e
OUT=${OUT:-gpurun_out/r06e}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "one" > $OUT/one_tests.log 2>&1 || { tail -40 $OUT/one_tests.log; exit 1; }
tail -1 $OUT/one_tests.log
MZH_DIAG_LIB=muzero-hanoi_amd/libmzh_diag.so timeout -k 10 120 python tools/one_stamps.py > $OUT/stamps.json
python -c "
import json;d=json.load(open('$OUT/stamps.json'));print(d['wave0_total'],d['sel_steps_per_sim'])
for w,v in d['ticks_per_sim'].items(): print(w, {k: round(x) for k, x in v.items()})"
timeout -k 10 300 python tools/one_probe.py --out $OUT/one_probe.json > $OUT/one_probe.log 2>&1 || { tail -20 $OUT/one_probe.log; exit 1; }
python -c "
import json;d=json.load(open('$OUT/one_probe.json'))
for r in d['rows']: print(r['disks'],r['sims'],r['roots'],'one %.3f coop %.3f'%(r['one_ms'],r['coop_ms']),r['identical'])
print(d['run_mcts'])"
timeout -k 10 300 python tools/bench_selfplay.py --legs drop-in --out $OUT/selfplay.json > $OUT/selfplay.log 2>&1 || { tail -20 $OUT/selfplay.log; exit 1; }
tail -1 $OUT/selfplay.log
