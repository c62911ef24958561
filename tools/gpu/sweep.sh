# profile sweep: for each bench workload the un-profiled bench line, rocprofv3 --kernel-trace --stats
# and separate PMC passes (tools/prof.sh), summarised and recorded under the profiled run's own key
# (tools/traffic.py), then the bench line re-run with the recorded traffic.
#   bash tools/gpu/sweep.sh "c2:" "b8192:--config 2 --shard 0/8" ...      (TAG:BENCH_ARGS pairs)
set -e
mkdir -p gpurun_out
for spec in "$@"; do
  T=${spec%%:*}
  A=${spec#*:}
  TAG=$T BENCH_ARGS="$A" bash tools/prof.sh > gpurun_out/sweep_$T.log 2>&1 || { tail -5 gpurun_out/sweep_$T.log; exit 1; }
  python tools/traffic.py gpurun_out $T --traffic-json gpurun_out/traffic_latest.json > gpurun_out/traffic_$T.json
  timeout -k 10 300 python bench.py $A --no-cpu-baseline --traffic-json gpurun_out/traffic_latest.json > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$T.json'));r=d['roofline'];print('$T','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel'],'%.4f'%r['kernel_ms'],'traffic',r['traffic'],'tree',r['tree']['frac'],(r['tree'].get('latency') or {}).get('frac'))"
done
