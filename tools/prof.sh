# rocprofv3 passes for the bench command: kernel trace + stats, then one PMC group per run
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Outputs under gpurun_out/prof_*.
# BENCH_ARGS adds bench.py options (default: the bench's own N=1 workload).
set -e
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
B="$R/bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS}"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_trace --output-format csv -- python3 $B > $R/gpurun_out/prof_trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/prof_hit --output-format csv -- python3 $B > $R/gpurun_out/prof_hit.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch --output-format csv -- python3 $B > $R/gpurun_out/prof_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/prof_write --output-format csv -- python3 $B > $R/gpurun_out/prof_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d $R/gpurun_out/prof_sq --output-format csv -- python3 $B > $R/gpurun_out/prof_sq.log 2>&1
cd $R
python3 tools/pmc_summary.py gpurun_out ${KERNEL:-mzh_wave_kernel} > gpurun_out/pmc_summary.json
cat gpurun_out/pmc_summary.json
