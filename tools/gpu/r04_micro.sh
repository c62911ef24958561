# round 4: price the MLP/tree overlap (tools/micro/overlap_probe.hip, built in-tree beforehand) and measure the
# dependent block-load latency; plus the 8,192- and 4,096-root bench lines with their caller-bounds legs
set -e
mkdir -p gpurun_out
timeout -k 10 300 tools/micro/overlap_probe > gpurun_out/overlap_probe.jsonl 2> gpurun_out/overlap_probe.err
cat gpurun_out/overlap_probe.jsonl
timeout -k 10 120 python bench.py --config 2 --shard 0/8 --no-cpu-baseline > gpurun_out/bench_8192.json 2> gpurun_out/bench_8192.err
timeout -k 10 120 python bench.py --config 1 --no-cpu-baseline > gpurun_out/bench_c1.json 2> gpurun_out/bench_c1.err
for b in 8192 c1; do python -c "import json;d=json.load(open('gpurun_out/bench_$b.json'));r=d['roofline'];print('$b','%.4e'%d['value'],'%.4f'%r['frac'],r['kernel'],r['kernel_ms'],'mm',r['with_minmax_in']['kernel'],r['with_minmax_in']['kernel_ms'])"; done
