# instruction mix of the search kernels (one rocprofv3 --pmc pass per counter group; each pass
# time-limited): bash tools/pmc_mix.sh "<bench args>" TAG
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
B="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-tree $1"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmcmix_$2_a --output-format csv -- python3 $B > $R/gpurun_out/pmcmix_$2_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d $R/gpurun_out/pmcmix_$2_b --output-format csv -- python3 $B > $R/gpurun_out/pmcmix_$2_b.log 2>&1
cd $R
python tools/pmc_kernel.py "${3:-_kernel<}" gpurun_out/pmcmix_$2_a gpurun_out/pmcmix_$2_b > gpurun_out/pmcmix_$2.json
cat gpurun_out/pmcmix_$2.json
