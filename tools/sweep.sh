set -e
mkdir -p gpurun_out
timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps.json 2>gpurun_out/stamps.err
timeout -k 10 120 python tools/phase_probe.py > gpurun_out/probe.json 2>/dev/null
for cfg in "4 50 4096" "4 50 8192" "4 50 16384" "4 50 65536" "4 200 16384" "7 100 32768" "3 25 8192"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --disks $1 --sims $2 --roots-per-gpu $3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_$1_$2_$3.json 2>>gpurun_out/bench_sweep.err
  python -c "import json;d=json.load(open('gpurun_out/bench_$1_$2_$3.json'));print('$cfg', '%.3e'%d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
