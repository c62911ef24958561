set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "search" > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
TAG=fl bash tools/prof.sh
MZH_LIB=$PWD/muzero-hanoi_amd/libmzh_base.so TAG=base bash tools/prof.sh
for t in base fl; do python tools/traffic.py gpurun_out $t > gpurun_out/traffic_$t.json; python - <<P
import json
d = json.load(open("gpurun_out/traffic_$t.json"))
for k in ("fused", "tree"):
    x = d[k]
    print("$t", k, x.get("avg_ns"), "read", x.get("hbm_read_bytes_corrected"), "write", x.get("hbm_write_bytes"), "l2hit", x.get("l2_hit_rate"))
P
done
