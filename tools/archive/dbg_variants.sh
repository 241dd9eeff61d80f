#!/bin/bash
# Build diagnostic variants of libyfm_hip.so into variants/ (git-ignored; they travel to the GPU box):
# yfm_kernels.hip recompiled with extra flags, linked with the regular objects of build/.
#   bash tools/archive/dbg_variants.sh <name> "<extra hipcc flags>"
set -eo pipefail
cd "$(dirname "$0")/.."
NAME=$1; EXTRA=$2
mkdir -p variants/obj
OBJ=variants/obj/yfm_kernels_$NAME.o
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -Iinclude $EXTRA \
  -c yieldfactormodels.jl_amd/csrc/yfm_kernels.hip -o $OBJ
OTHERS=$(ls yieldfactormodels.jl_amd/build/*.o | grep -v yfm_kernels.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OTHERS $OBJ -o variants/libyfm_$NAME.so
echo variants/libyfm_$NAME.so
