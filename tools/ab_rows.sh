set -e
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
for R in 32 16; do
  MZH_ROWS=$R timeout -k 10 120 python tools/phase_probe.py > gpurun_out/probe_R$R.json 2>/dev/null
  MZH_ROWS=$R timeout -k 10 120 python tools/phase_probe.py --roots 16384 > gpurun_out/probe_R${R}_16k.json 2>/dev/null
done
tail -2 gpurun_out/gpu_tests.log
cat gpurun_out/probe_R*.json
