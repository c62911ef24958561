# build libmzh_<tag>.so from the csrc/ + include/ of a git revision (A/B against older kernels on one box)
#   bash tools/build_rev.sh <rev> <tag>      e.g. bash tools/build_rev.sh HEAD base
set -e
REV=$1; TAG=$2
R=$(cd "$(dirname "$0")/.." && pwd)
D=/tmp/mzh_rev_$TAG
rm -rf $D && mkdir -p $D
git -C $R archive $REV muzero-hanoi_amd/csrc include | tar -x -C $D
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I $D/include"
for s in mzh_api mzh_search mzh_wave mzh_env mzh_train; do
  /opt/rocm/bin/hipcc $FL -c $D/muzero-hanoi_amd/csrc/$s.hip -o $D/$s.o &
done
wait
printf 'static const char kId[] = "MZH_BUILD_ID:rev-%s";\nextern "C" const char* mzh_build_id(void) { return kId + 13; }\n' $TAG > $D/id.cpp
g++ -O2 -fPIC -c $D/id.cpp -o $D/id.o
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $D/*.o -o $R/muzero-hanoi_amd/libmzh_$TAG.so -Wl,-rpath,/opt/rocm/lib
echo $R/muzero-hanoi_amd/libmzh_$TAG.so
