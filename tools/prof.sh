# rocprofv3 passes for the bench command: kernel trace + stats, then separate PMC passes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).  Outputs under gpurun_out/prof_*.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace --output-format csv -- python $B > gpurun_out/prof_trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/prof_hit --output-format csv -- python $B > gpurun_out/prof_hit.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_fetch --output-format csv -- python $B > gpurun_out/prof_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_write --output-format csv -- python $B > gpurun_out/prof_write.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d gpurun_out/prof_sq --output-format csv -- python $B > gpurun_out/prof_sq.log 2>&1 || true
find gpurun_out/prof_* -name "*.csv" | head -50
