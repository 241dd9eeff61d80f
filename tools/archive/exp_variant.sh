#!/bin/bash
# Build an experiment variant of libyfm_hip.so into variants/: the listed translation units recompiled with
# extra flags, linked with the regular objects of build/ (git-ignored; travels to the GPU box).
#   bash tools/archive/exp_variant.sh <name> "<extra hipcc flags>" <tu> [<tu> ...]     (tu: yfm_kernels, yfm_capi, …)
set -eo pipefail
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=$2; shift 2
mkdir -p variants/obj
objs=""
for tu in "$@"; do
  o=variants/obj/${tu}_$NAME.o
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -mllvm -amdgpu-spill-vgpr-to-agpr=0 -Iinclude $EXTRA -c yieldfactormodels.jl_amd/csrc/$tu.hip -o $o &
  objs="$objs $o"
done
wait
others=$(ls yieldfactormodels.jl_amd/build/*.o | grep -v -E "/($(echo "$@" | tr ' ' '|'))\.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $others $objs -o variants/libyfm_$NAME.so
echo variants/libyfm_$NAME.so
