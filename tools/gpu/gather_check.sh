# the result all_gather on the GPU: 2-rank gloo rehearsal of the sharded bench (even shards) + smoke
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || exit $?
tail -c 400 gpurun_out/bench_gloo2.json
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()"
