#!/bin/bash
# kernel trace of the pipelined drop-in self-play loop (search / env kernel durations and the gaps between them)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/dropin_trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/dropin_trace -o run -- \
  python3 $R/tools/dropin_profile.py --seconds 2 > $R/gpurun_out/dropin_trace.log 2>&1 || { tail -5 $R/gpurun_out/dropin_trace.log; exit 1; }
head -3 $R/gpurun_out/dropin_trace.log
