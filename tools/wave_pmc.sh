# PMC passes (one counter group per run, each killed at 60 s) for the wave kernel at the metric batch
set -e
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
B="$R/bench.py --roots-per-gpu 65536 --steps 2 --warmup 1 --no-cpu-baseline --kernel wave"
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $R/gpurun_out/pmc_a --output-format csv -- python3 $B > $R/gpurun_out/pmc_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $R/gpurun_out/pmc_b --output-format csv -- python3 $B > $R/gpurun_out/pmc_b.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM -d $R/gpurun_out/pmc_c --output-format csv -- python3 $B > $R/gpurun_out/pmc_c.log 2>&1
find $R/gpurun_out/pmc_* -name "*counter_collection.csv"
