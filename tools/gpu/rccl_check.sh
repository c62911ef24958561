# RCCL on the box's GPU (world size 1, tests/test_gpu_rccl.py), then the N=8 bench command form
# rehearsed with 8 gloo ranks sharing the one GPU (bench.py self-launches the ranks; timing meaningless)
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/rccl_test.log 2>&1 || { tail -40 gpurun_out/rccl_test.log; exit 1; }
tail -3 gpurun_out/rccl_test.log
timeout -k 10 400 python bench.py --gpus 8 --dist-backend gloo --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_gloo8.json 2> gpurun_out/bench_gloo8.err || { tail -30 gpurun_out/bench_gloo8.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_gloo8.json'));print(d['n_gpus'],d['value'],d['dist'])"
