# VALU instruction mix of the fused wave kernel and its tree-only replay instantiation at configs[2]
# (65,536 roots): two PMC passes of the bench command, per-kernel means (tools/pmc_kernel.py)
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-minmax-leg"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT -d $R/gpurun_out/valu_a --output-format csv -- python3 $B > $R/gpurun_out/valu_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d $R/gpurun_out/valu_b --output-format csv -- python3 $B > $R/gpurun_out/valu_b.log 2>&1
cd $R
python tools/pmc_kernel.py "mzh_wave_kernel<2, false" gpurun_out/valu_a gpurun_out/valu_b > gpurun_out/valu_fused.json
python tools/pmc_kernel.py "mzh_wave_kernel<2, true" gpurun_out/valu_a gpurun_out/valu_b > gpurun_out/valu_tree.json
cat gpurun_out/valu_fused.json gpurun_out/valu_tree.json
