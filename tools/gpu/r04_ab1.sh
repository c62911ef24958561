# HISTORICAL (record of profiles/r04_experiments.json): the 8-wave / phase-locked / priority variants it
# compares were removed from the sources after the measurement (commit 83d898f); it no longer runs as written.
# A/B: wave kernel 4-wave (drifting) vs 8-wave phase-locked workgroups; cooperative 32-root tile on 4 vs 8 waves
set -e
mkdir -p gpurun_out
B="timeout -k 10 300 python bench.py --no-cpu-baseline --no-tree --no-minmax-leg --steps 10 --warmup 2"
show() { python -c "import json,sys;d=json.load(open('$1'));r=d['roofline'];print('$1',r['kernel'],'%.4f ms'%r['kernel_ms'],'frac %.4f'%r['frac'])"; }
for rep in 1 2; do
  for wg in 4 8; do
    MZH_WAVE_WG=$wg $B > gpurun_out/ab_wg${wg}_c2_$rep.json 2> gpurun_out/ab.err && show gpurun_out/ab_wg${wg}_c2_$rep.json
    MZH_WAVE_WG=$wg $B --config 2 --shard 0/2 > gpurun_out/ab_wg${wg}_s32k_$rep.json 2>> gpurun_out/ab.err && show gpurun_out/ab_wg${wg}_s32k_$rep.json
    MZH_WAVE_WG=$wg $B --config 4 --steps 4 > gpurun_out/ab_wg${wg}_c4_$rep.json 2>> gpurun_out/ab.err && show gpurun_out/ab_wg${wg}_c4_$rep.json
  done
  for cw in 4 8; do
    MZH_COOP_WAVES=$cw $B --config 2 --shard 0/8 > gpurun_out/ab_cw${cw}_s8k_$rep.json 2>> gpurun_out/ab.err && show gpurun_out/ab_cw${cw}_s8k_$rep.json
  done
done
MZH_WAVE_WG=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_parity_corners.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "wave and (large_batch or full_size or sharded or agreement or deep or replay_vs)" > gpurun_out/ab_wg8_tests.log 2>&1; tail -2 gpurun_out/ab_wg8_tests.log
MZH_COOP_WAVES=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu -k "full_size or sharded or caller_bounds" > gpurun_out/ab_cw8_tests.log 2>&1; tail -2 gpurun_out/ab_cw8_tests.log
