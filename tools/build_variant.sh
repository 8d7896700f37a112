#!/bin/bash
# Build an A/B variant of the library outside the product tree. The shipped sources carry
# no A/B knobs: a variant is a patch against celestia-app_amd/csrc (paths as `git diff`
# prints them) applied to a copy of the sources, plus optional extra compile flags:
#   bash tools/build_variant.sh <name> [<patch file> | -] ["<flags>"]  ->  variants/lib<name>.so
# (tools/gpu_ab.sh times variants on the GPU box; build_variants/ and variants/ are
# git-ignored.)
set -e
name=$1; patch=${2:--}; flags=$3
[ "$patch" != "-" ] && patch=$(realpath "$patch")
cd "$(dirname "$0")/.."
bd=build_variants/$name
rm -rf $bd
mkdir -p $bd/src variants
cp -r celestia-app_amd/csrc $bd/src/csrc
cp -r include $bd/include
if [ "$patch" != "-" ]; then
  # the patch names a/celestia-app_amd/csrc/<file> (git diff form): strip two components
  (cd $bd/src && patch -p2 --quiet < "$patch")
fi
HIPCC=/opt/rocm/bin/hipcc
# the library's sources, as the Makefile lists them
srcs=$(sed -n 's/^SRC := //p' celestia-app_amd/Makefile | sed 's#csrc/##g')
objs=""
for f in $srcs; do
  extra=""
  [ "$f" = nmt_kernels.hip ] && extra="-mllvm -amdgpu-sched-strategy=max-memory-clause"
  $HIPCC --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $extra $flags -x hip \
    -I$bd/include -c $bd/src/csrc/$f -o $bd/$f.o &
  objs="$objs $bd/$f.o"
done
wait
$HIPCC --offload-arch=gfx950 -shared -o variants/lib$name.so $objs -L/opt/rocm/lib -lrocprofiler-sdk-roctx -ldl \
  -Wl,-rpath,/opt/rocm/lib
echo variants/lib$name.so
