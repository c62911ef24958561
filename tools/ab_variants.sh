# A/B the diagnostic variants: phase stamps for libmzh_diag.so and every libmzh_diag_<tag>.so
set -e
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in muzero-hanoi_amd/libmzh_diag*.so; do
  tag=$(basename "$lib" .so | sed 's/libmzh_diag//; s/^_//'); tag=${tag:-base}
  MZH_DIAG_LIB=$PWD/$lib timeout -k 10 200 python tools/stamp_probe.py > gpurun_out/stamps_$tag.json
  python - "$tag" <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/stamps_{t}.json"))
tot = d["search_per_sim_total"]
print(t, "per-sim ticks", [round(x) for x in tot], "select-level", d["select_level_ticks"])
PY
done
