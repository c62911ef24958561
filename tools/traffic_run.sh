# parity suite, then rocprofv3 stats + PMC passes of the default bench (65,536 roots: fused + replay kernels)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
TAG=${TAG:-cur} BENCH_ARGS="${BENCH_ARGS:-}" bash tools/prof.sh
python tools/traffic.py gpurun_out ${TAG:-cur} > gpurun_out/traffic_${TAG:-cur}.json
python - <<P
import json
d = json.load(open("gpurun_out/traffic_${TAG:-cur}.json"))
for k in ("fused", "tree"):
    x = d[k]
    print(k, x.get("avg_ns"), "read", x.get("hbm_read_bytes_corrected"), "write", x.get("hbm_write_bytes"), "l2hit", x.get("l2_hit_rate"), "mfma", x.get("mfma_busy_frac"))
P
