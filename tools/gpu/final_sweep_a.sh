# final pass, part A: GPU tests + smoke + the driver's default bench + gloo2 rehearsal (tools/gpu/final.sh),
# then on the same lease the headline's rocprofv3 stats + PMC passes and the two small-batch workloads
set -e
bash tools/gpu/final.sh
bash tools/gpu/sweep.sh "c2:" "b8192:--config 2 --shard 7/8" "c1:--config 1"
