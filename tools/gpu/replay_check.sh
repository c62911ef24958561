#!/bin/bash
# device replay draw: GPU tests of the draw / write-back and the training-update bench legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_replay.py tests/test_training.py > gpurun_out/replay_tests.txt 2>&1 || { tail -30 gpurun_out/replay_tests.txt; exit 1; }
tail -3 gpurun_out/replay_tests.txt
timeout -k 10 300 python -u tools/bench_train.py --legs fused,fused-hostdraw,graph --out gpurun_out/replay_train_bench.json \
  > gpurun_out/replay_train_bench.log 2>&1 || { tail -30 gpurun_out/replay_train_bench.log; exit 1; }
cat gpurun_out/replay_train_bench.log
