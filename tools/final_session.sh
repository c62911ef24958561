# end-of-session GPU pass: parity suite, rocprofv3 stats + PMC at 8,192 / 4,096 roots, bench lines at
# every BASELINE config on one GPU (default = configs[2] with the CPU baseline) + a 2-rank gloo rehearsal
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
TAG=b8192 BENCH_ARGS="--roots-per-gpu 8192" bash tools/prof.sh
TAG=c1 BENCH_ARGS="--config 1" bash tools/prof.sh
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
cat gpurun_out/bench_default.json
for C in 1 3 4; do
  timeout -k 10 200 python bench.py --config $C --no-cpu-baseline > gpurun_out/bench_c$C.json 2> gpurun_out/bench_c$C.err
  cat gpurun_out/bench_c$C.json
done
timeout -k 10 120 python bench.py --roots-per-gpu 8192 --no-cpu-baseline > gpurun_out/bench_8192.json 2> gpurun_out/bench_8192.err
cat gpurun_out/bench_8192.json
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
cat gpurun_out/bench_gloo2.json
