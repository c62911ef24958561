# final pass, part C: the secondary rows (self-play, evaluation, training updates; tools/gpu/secondary.sh), the
# scalar env step, and the latency path -- crossover probe + run_mcts under rocprofv3 --kernel-trace --stats (the
# latency kernel's own launch durations), then its phase stamps on the diagnostic build; the replay draw's stamps
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
mkdir -p gpurun_out
bash tools/gpu/secondary.sh
timeout -k 10 300 python tools/bench_env.py --out gpurun_out/env_bench.json > gpurun_out/env_bench.log 2>&1 || { tail -20 gpurun_out/env_bench.log; exit 1; }
grep leg gpurun_out/env_bench.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_one --output-format csv -- python3 $R/tools/one_probe.py --out $R/gpurun_out/one_probe.json > $R/gpurun_out/prof_one.log 2>&1
cd $R
tail -2 gpurun_out/prof_one.log
MZH_DIAG_LIB=muzero-hanoi_amd/libmzh_diag.so timeout -k 10 120 python tools/one_stamps.py > gpurun_out/one_stamps.json
python -c "import json;d=json.load(open('gpurun_out/one_stamps.json'));print('stamps',d['wave0_total'])"
# the device replay draw: its phase stamps (diagnostic build) and the fused update's host-side split
MZH_LIB=muzero-hanoi_amd/libmzh_diag.so timeout -k 10 120 python tools/replay_stamps.py --out gpurun_out/replay_stamps.json
timeout -k 10 200 python tools/train_host_profile.py --out gpurun_out/train_host_profile.json
