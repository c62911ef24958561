# the secondary measurements on the current build: self-play decisions/s, batched
# evaluation, training updates/s -- each with its host-CPU leg
set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_selfplay.py --legs batched,batched-legacy,drop-in,cpu --out gpurun_out/selfplay.json > gpurun_out/selfplay.log 2>&1 || { tail -20 gpurun_out/selfplay.log; exit 1; }
tail -3 gpurun_out/selfplay.log
timeout -k 10 300 python tools/bench_eval.py --out gpurun_out/eval.json > gpurun_out/eval.log 2>&1 || { tail -20 gpurun_out/eval.log; exit 1; }
tail -3 gpurun_out/eval.log
timeout -k 10 300 python tools/bench_train.py --out gpurun_out/train.json > gpurun_out/train.log 2>&1 || { tail -20 gpurun_out/train.log; exit 1; }
tail -3 gpurun_out/train.log
