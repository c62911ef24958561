# rocprofv3 passes for one bench command: kernel trace + stats, then one PMC group per run (FETCH_SIZE
# and WRITE_SIZE cannot share a pass on gfx950; each pass killed at 120 s).  Outputs under
# gpurun_out/prof_<TAG>_*; BENCH_ARGS adds bench.py options (default: the bench's own N=1 workload).
#   TAG=c2 BENCH_ARGS="" bash tools/prof.sh ; python tools/traffic.py gpurun_out c2 --traffic-json gpurun_out/traffic_latest.json
set -e
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
T=${TAG:-run}
export TMPDIR=/tmp
mkdir -p gpurun_out
B="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS}"
# the same command un-profiled first (same box and build: the HIP-event time the profile is compared with)
timeout -k 10 300 python3 $B > $R/gpurun_out/prof_${T}_plain.json 2> $R/gpurun_out/prof_${T}_plain.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_${T}_trace --output-format csv -- python3 $B > $R/gpurun_out/prof_${T}_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/prof_${T}_hit --output-format csv -- python3 $B > $R/gpurun_out/prof_${T}_hit.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_${T}_fetch --output-format csv -- python3 $B > $R/gpurun_out/prof_${T}_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_${T}_write --output-format csv -- python3 $B > $R/gpurun_out/prof_${T}_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $R/gpurun_out/prof_${T}_sq --output-format csv -- python3 $B > $R/gpurun_out/prof_${T}_sq.log 2>&1
cd $R
tail -1 gpurun_out/prof_${T}_trace.log
