# parity suite + the bench line at every BASELINE config on one GPU (+ a 2-rank gloo rehearsal of N>1)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
cat gpurun_out/bench_default.json
for C in 1 3 4; do
  timeout -k 10 200 python bench.py --config $C --no-cpu-baseline > gpurun_out/bench_c$C.json 2> gpurun_out/bench_c$C.err
  cat gpurun_out/bench_c$C.json
done
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
cat gpurun_out/bench_gloo2.json
