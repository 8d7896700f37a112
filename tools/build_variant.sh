#!/bin/bash
# Build an A/B variant of the library with extra compile flags, outside the product tree:
#   bash tools/build_variant.sh <name> "<flags>"   ->  variants/lib<name>.so
# (tools/gpu_variants.sh times variants on the GPU box; variants/ is git-ignored.)
set -e
cd "$(dirname "$0")/.."
name=$1; flags=$2
bd=build_variants/$name
mkdir -p $bd variants
HIPCC=/opt/rocm/bin/hipcc
srcs="api.cpp square.cpp proof.cpp inclusion.cpp inclusion_paths.cpp rs_kernels.hip rs_bitslice.hip rs_axis.hip rs_decode_axis.hip rs_decode_gf16.hip rs_gf16x.hip nmt_kernels.hip repair_kernels.hip"
objs=""
for f in $srcs; do
  extra=""
  [ "$f" = nmt_kernels.hip ] && extra="-mllvm -amdgpu-sched-strategy=max-memory-clause"
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $extra $flags -x hip \
    -c celestia-app_amd/csrc/$f -o $bd/$f.o &
  objs="$objs $bd/$f.o"
done
wait
$HIPCC --offload-arch=gfx950 -shared -o variants/lib$name.so $objs -L/opt/rocm/lib -lrocprofiler-sdk-roctx \
  -Wl,-rpath,/opt/rocm/lib
echo variants/lib$name.so
