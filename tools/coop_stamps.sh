# phase stamps of the cooperative search kernel at 8,192 / 4,096 roots (needs libmzh_diag.so: python -m muzero_hanoi_amd.build --diag)
set -e
mkdir -p gpurun_out
for B in 8192 4096; do timeout -k 10 120 python tools/stamp_probe.py $B > gpurun_out/stamps_$B.json; done
python - <<'P'
import json
for B in (8192, 4096):
    d = json.load(open(f"gpurun_out/stamps_{B}.json"))
    print(B, {k: round(sum(v)/4) for k, v in d["search_per_sim"].items()}, "levels", [round(x,2) for x in d["select_levels_per_sim"]], d["select_level_ticks"])
P
