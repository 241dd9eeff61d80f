#!/bin/bash
# Build tools/variants/<tag>.so: the in-tree objects with <file.hip> (a modified copy of one csrc translation unit)
# compiled in place of its namesake.  usage: bash tools/r6/variant.sh <tag> <path/to/yfm_xxx.hip> [extra flags]
set -e
TAG=$1; SRC=$2; shift 2
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
B=$ROOT/yieldfactormodels.jl_amd/build
STEM=$(basename "$SRC" .hip)
mkdir -p $ROOT/tools/variants
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -mllvm -amdgpu-spill-vgpr-to-agpr=0 -I$ROOT/include -I$ROOT/yieldfactormodels.jl_amd/csrc"
/opt/rocm/bin/hipcc $FLAGS "$@" -x hip -c "$SRC" -o $ROOT/tools/variants/${TAG}_$STEM.o
OBJS=""
for o in $B/*.o; do
  if [ "$(basename $o .o)" = "$STEM" ]; then OBJS="$OBJS $ROOT/tools/variants/${TAG}_$STEM.o"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o $ROOT/tools/variants/$TAG.so
rm -f $ROOT/tools/variants/${TAG}_$STEM.o
echo $ROOT/tools/variants/$TAG.so
