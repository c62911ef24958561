# search parity tests (tests/test_gpu_parity.py -k search) against every libmzh_<tag>.so fast variant
set -e
mkdir -p gpurun_out
for lib in muzero-hanoi_amd/libmzh_[a-z]*.so; do
  case "$lib" in *diag*) continue;; esac
  tag=$(basename "$lib" .so)
  MZH_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "search" > gpurun_out/parity_$tag.log 2>&1 || { echo "$tag FAILED"; tail -20 gpurun_out/parity_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/parity_$tag.log)"
done
