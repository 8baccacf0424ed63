# Development aid for A/B timing: build the device code of a git revision (default HEAD)
# into fscl_amd/_build_<name> against the current host objects.
#   bash tools/build_ref_variant.sh [rev] [name] [extra hipcc flags...]
set -e
REV=${1:-HEAD}; NAME=${2:-head}; shift $(( $# > 2 ? 2 : $# )) || true
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
mkdir -p $T/fscl_amd/csrc/device
git -C $R show $REV:fscl_amd/csrc/device/fsclg.hip > $T/fscl_amd/csrc/device/fsclg.hip
ln -s $R/include $T/include
OUT=$R/fscl_amd/_build_$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Wno-unused-value -mllvm -amdgpu-sched-strategy=iterative-ilp \
  -Wno-unused-result "$@" -c $T/fscl_amd/csrc/device/fsclg.hip -o $OUT/fsclg.o
g++ -shared -o $OUT/libfscl_amd.so $R/fscl_amd/_build/{util,input,spectrum,tables,scan,ranks}.o $OUT/fsclg.o \
  -L/opt/rocm/lib -lamdhip64 -lgomp -lm -lpthread -Wl,-rpath,/opt/rocm/lib
rm -rf $T
echo $OUT/libfscl_amd.so
