# latency-kernel phase stamps (diagnostic builds: unroll 2 / 8 / 16 of the K = 256 chains)
set -e
mkdir -p gpurun_out/r06c
for v in "" _u8 _u16; do
  MZH_DIAG_LIB=muzero-hanoi_amd/libmzh_diag$v.so timeout -k 10 120 python tools/one_stamps.py > gpurun_out/r06c/stamps$v.json
  python -c "import json;d=json.load(open('gpurun_out/r06c/stamps$v.json'));print('$v',d['wave0_total'],d['sel_steps_per_sim'],d['ticks_per_sim']['wave0'])"
done
MZH_DIAG_LIB=muzero-hanoi_amd/libmzh_diag.so timeout -k 10 120 python tools/one_stamps.py --disks 4 --sims 50 > gpurun_out/r06c/stamps_n4.json
python -c "import json;d=json.load(open('gpurun_out/r06c/stamps_n4.json'));print('n4',d['wave0_total'],d['sel_steps_per_sim'],d['ticks_per_sim']['wave0'])"
