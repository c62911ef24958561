# final pass, part B: rocprofv3 stats + PMC of every other bench workload (tools/gpu/sweep.sh)
set -e
bash tools/gpu/sweep.sh "s16k:--config 2 --shard 3/4" "s32k:--config 2 --shard 1/2" "c3:--config 3" "c4:--config 4" "c4s8:--config 4 --shard 0/8"
