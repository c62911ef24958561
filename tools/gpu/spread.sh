# run-to-run spread of the default bench line on one box (three back-to-back runs, no CPU baseline)
set -e
mkdir -p gpurun_out
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/spread_$r.json 2> gpurun_out/spread_$r.err
  python -c "import json;d=json.load(open('gpurun_out/spread_$r.json'));print('run $r','%.4e'%d['value'],'%.4f'%d['roofline']['frac'],'%.4f ms'%d['roofline']['kernel_ms'])"
done
