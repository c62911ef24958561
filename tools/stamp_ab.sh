# phase stamps of the cooperative kernel for two diagnostic builds (A/B): fused search at 8,192 and
# 4,096 roots and the replay (tree-only) instantiation at 8,192
#   LIBS="muzero-hanoi_amd/libmzh_diag_old.so muzero-hanoi_amd/libmzh_diag.so" bash tools/stamp_ab.sh
set -e
mkdir -p gpurun_out
for L in ${LIBS:-muzero-hanoi_amd/libmzh_diag.so}; do
  t=$(basename $L .so)
  for B in 8192 4096; do MZH_DIAG_LIB=$L timeout -k 10 120 python tools/stamp_probe.py $B > gpurun_out/stamps_${t}_$B.json; done
  MZH_DIAG_LIB=$L timeout -k 10 120 python tools/stamp_probe.py 8192 --replay > gpurun_out/stamps_${t}_8192r.json
done
python - <<'P'
import json, os
for L in os.environ.get("LIBS", "muzero-hanoi_amd/libmzh_diag.so").split():
    t = os.path.basename(L)[:-3]
    for B in ("8192", "4096", "8192r"):
        d = json.load(open(f"gpurun_out/stamps_{t}_{B}.json"))
        print(t, B, {k.split(":")[0]: round(sum(v)/4) for k, v in d["search_per_sim"].items()}, "tot", round(sum(d["search_per_sim_total"])/4), "lv", [round(x,2) for x in d["select_levels_per_sim"]])
P
