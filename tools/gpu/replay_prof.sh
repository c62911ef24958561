#!/bin/bash
# kernel durations of the device replay draw inside the fused training-update loop
set -o pipefail
mkdir -p gpurun_out/replay_prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/replay_prof -o run --output-format csv -- \
  python3 $GRAFT_REPO_ROOT/tools/bench_train.py --legs fused --steps 100 > $GRAFT_REPO_ROOT/gpurun_out/replay_prof.log 2>&1 \
  || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/replay_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/replay_prof -name "*kernel_stats.csv" -exec cat {} \;
