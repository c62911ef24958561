# search parity tests (tests/test_gpu_parity.py -k search) against the named fast variants:
#   bash tools/variant_parity.sh TAG [TAG ...]     (muzero-hanoi_amd/libmzh_<TAG>.so, built with
#   python -m muzero_hanoi_amd.build --fast-variant=TAG=DEF1,DEF2); each log line names the build flags
set -e
mkdir -p gpurun_out
for tag in "$@"; do
  lib=muzero-hanoi_amd/libmzh_$tag.so
  echo "$tag: $(stat -c %y $lib) flags: $(cat $lib.flags)"
  MZH_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "search" > gpurun_out/parity_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 gpurun_out/parity_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/parity_$tag.log)"
done
