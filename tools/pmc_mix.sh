# instruction mix and wait split of the search kernels (one rocprofv3 --pmc pass per counter group; each
# pass time-limited): bash tools/pmc_mix.sh "<bench args>" TAG ["kernel name substring"]
#   a: instruction counts; b: issue / wait cycles (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES);
#   c: in-flight vector-memory / LDS instruction levels (Little's law: level / count = mean latency)
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
export TMPDIR=/tmp
mkdir -p $R/gpurun_out
B="$R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-minmax-leg $1"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/pmcmix_$2_a --output-format csv -- python3 $B > $R/gpurun_out/pmcmix_$2_a.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES -d $R/gpurun_out/pmcmix_$2_b --output-format csv -- python3 $B > $R/gpurun_out/pmcmix_$2_b.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $R/gpurun_out/pmcmix_$2_c --output-format csv -- python3 $B > $R/gpurun_out/pmcmix_$2_c.log 2>&1 || echo "pass c failed (counters unavailable?)"
cd $R
python tools/pmc_kernel.py "${3:-_kernel<}" gpurun_out/pmcmix_$2_a gpurun_out/pmcmix_$2_b gpurun_out/pmcmix_$2_c > gpurun_out/pmcmix_$2.json
cat gpurun_out/pmcmix_$2.json
