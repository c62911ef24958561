set -e
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for k in split coop; do
B="$R/bench.py --roots-per-gpu 8192 --steps 3 --warmup 1 --no-cpu-baseline --no-tree --kernel $k"
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY -d $R/gpurun_out/pmc/${k}_a --output-format csv -- python3 $B > $R/gpurun_out/pmc/${k}_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d $R/gpurun_out/pmc/${k}_b --output-format csv -- python3 $B > $R/gpurun_out/pmc/${k}_b.log 2>&1
cd $R
done
find gpurun_out/pmc -name "*counter_collection.csv" | head
