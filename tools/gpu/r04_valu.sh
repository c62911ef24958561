# VALU instruction mix of the fused wave kernel and its tree-only replay instantiation at the given workload
# (65,536 roots): two PMC passes of the bench command, per-kernel means (tools/pmc_kernel.py)
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-minmax-leg ${BENCH_ARGS}"; T=${TAG:-c2}; K=${KPAT:-mzh_wave_kernel<2}
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT -d $R/gpurun_out/valu_${T}_a --output-format csv -- python3 $B > $R/gpurun_out/valu_${T}_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d $R/gpurun_out/valu_${T}_b --output-format csv -- python3 $B > $R/gpurun_out/valu_${T}_b.log 2>&1
cd $R
python tools/pmc_kernel.py "${K}, false" gpurun_out/valu_${T}_a gpurun_out/valu_${T}_b > gpurun_out/valu_${T}_fused.json
python tools/pmc_kernel.py "${K}, true" gpurun_out/valu_${T}_a gpurun_out/valu_${T}_b > gpurun_out/valu_${T}_tree.json
cat gpurun_out/valu_${T}_fused.json gpurun_out/valu_${T}_tree.json
